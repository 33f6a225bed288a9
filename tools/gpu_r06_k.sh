#!/bin/bash
# Round-6 GPU pass K: fp32 cut pass at 3 blocks per CU (logs stored at once) against 2 blocks per CU
# (logs' first entries held in a register, no spills): storm driver protocol and ssn; cut tests.
set -u
mkdir -p gpurun_out
S="--instance ssn --scenarios 100000 --vertices 16384"
bash tools/ab_bench.sh r06k "" "TWOSD_LIB=h2" "$S" "TWOSD_LIB=h2 $S" || exit 1
cat gpurun_out/r06k.txt
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_cut.py tests/test_gpu_large_v.py tests/test_gpu_configs.py > gpurun_out/r06k_tests.log 2>&1 || { tail -30 gpurun_out/r06k_tests.log; exit 1; }
tail -1 gpurun_out/r06k_tests.log
TWOSD_LIB=h2 timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_cut.py tests/test_gpu_large_v.py > gpurun_out/r06k_tests_h2.log 2>&1 || { tail -30 gpurun_out/r06k_tests_h2.log; exit 1; }
tail -1 gpurun_out/r06k_tests_h2.log

#!/bin/bash
# Round-6 GPU pass H: the fp32 cut pass with the wave-wide no-log test, at 2 and 3 blocks per CU
# (storm driver protocol and ssn |V| = 16384), then the cut parity tests on the default build.
set -u
S="--instance ssn --scenarios 100000 --vertices 16384"
bash tools/ab_bench.sh r06h "" "TWOSD_LIB=b3" "$S" "TWOSD_LIB=b3 $S" || exit 1
cat gpurun_out/r06h.txt
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_cut.py tests/test_gpu_large_v.py tests/test_gpu_configs.py > gpurun_out/r06h_tests.log 2>&1 || { tail -30 gpurun_out/r06h_tests.log; exit 1; }
tail -1 gpurun_out/r06h_tests.log

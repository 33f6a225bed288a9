#!/bin/bash
# Round-6 GPU pass E: the fp32 MFMA cut pass -- cut parity tests (both passes, the fallback), the
# iteration replay and the per-rank config tests, then the storm driver protocol with the fp32 pass
# (default) and the fp64 pass (TWOSD_CUT_F32=0), and ssn |V| = 16384.
set -u
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_cut.py tests/test_gpu_large_v.py tests/test_gpu_julia_mirror.py tests/test_gpu_configs.py tests/test_gpu_dist.py > gpurun_out/r06e_tests.log 2>&1 || { tail -40 gpurun_out/r06e_tests.log; exit 1; }
tail -2 gpurun_out/r06e_tests.log
bash tools/ab_bench.sh r06e "" "TWOSD_CUT_F32=0" "--instance ssn --scenarios 100000 --vertices 16384" "TWOSD_CUT_F32=0 --instance ssn --scenarios 100000 --vertices 16384" || exit 1
cat gpurun_out/r06e.txt

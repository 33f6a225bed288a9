#!/bin/bash
# Round-5 GPU pass E: cut parity tests, the cut alone at 1M (fixup stamps variant, then the
# default build), the storm warm-start hindsight table at x_EV.
set -u
mkdir -p gpurun_out
echo "cut tests"
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_cut.py tests/test_gpu_large_v.py tests/test_gpu_julia_mirror.py > gpurun_out/r05e_tests.log 2>&1 || { tail -30 gpurun_out/r05e_tests.log; exit 1; }
tail -2 gpurun_out/r05e_tests.log
echo "cut speed"
TWOSD_LIB=fxst TWOSD_FIX_STAMPS_PRINT=1 timeout -k 10 200 python3 -u tools/cut_speed.py 1000000 4096 3 || exit 1
timeout -k 10 200 python3 -u tools/cut_speed.py 1000000 4096 5 || exit 1
echo "storm hindsight at x_EV"
timeout -k 10 600 python3 -u tools/ssn_hindsight.py 96 16 0 storm > gpurun_out/r05e_storm_hindsight.txt 2> gpurun_out/r05e_storm.err || { tail -3 gpurun_out/r05e_storm.err; exit 1; }
cat gpurun_out/r05e_storm_hindsight.txt

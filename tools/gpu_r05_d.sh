#!/bin/bash
# Round-5 GPU pass D: cut parity tests, the cut alone at 1M (twins kept vs left out), a kernel
# trace of the driver's bench command, the ssn warm-start hindsight table.
set -u
mkdir -p gpurun_out
echo "cut tests"
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_cut.py tests/test_gpu_large_v.py tests/test_gpu_julia_mirror.py > gpurun_out/r05d_tests.log 2>&1 || { tail -30 gpurun_out/r05d_tests.log; exit 1; }
tail -2 gpurun_out/r05d_tests.log
echo "cut speed"
TWOSD_CUT_TWINS=0 timeout -k 10 200 python3 -u tools/cut_speed.py 1000000 4096 5 || exit 1
timeout -k 10 200 python3 -u tools/cut_speed.py 1000000 4096 5 || exit 1
echo "trace"
bash tools/prof_trace.sh r05_tr2 || exit 1
echo "hindsight"
timeout -k 10 500 python3 -u tools/ssn_hindsight.py 500 16 > gpurun_out/r05d_ssn_hindsight.txt 2> gpurun_out/r05d_ssn.err || { tail -3 gpurun_out/r05d_ssn.err; exit 1; }
cat gpurun_out/r05d_ssn_hindsight.txt
echo "storm hindsight at x_EV"
timeout -k 10 400 python3 -u tools/ssn_hindsight.py 160 16 0 storm > gpurun_out/r05d_storm_hindsight.txt 2> gpurun_out/r05d_storm.err || { tail -3 gpurun_out/r05d_storm.err; exit 1; }
cat gpurun_out/r05d_storm_hindsight.txt

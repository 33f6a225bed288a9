#!/bin/bash
# Round-6 GPU pass U: solve_push's full mode (every dual recovered in the main pass, representatives
# gathered) -- the push tests, then the ssn |V| = 16384 config and the storm driver protocol with the
# automatic choice against TWOSD_PUSH_MODE=1 (always re-solve).
set -u
mkdir -p gpurun_out/r06u
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_vkey.py > gpurun_out/r06u/tests.log 2>&1 || { tail -30 gpurun_out/r06u/tests.log; exit 1; }
tail -1 gpurun_out/r06u/tests.log
bash tools/ab_bench.sh r06u/ab "--instance ssn --scenarios 100000 --vertices 16384" "TWOSD_PUSH_MODE=1 --instance ssn --scenarios 100000 --vertices 16384" "" "TWOSD_PUSH_MODE=1" || exit 1

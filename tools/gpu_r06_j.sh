#!/bin/bash
# Round-6 GPU pass J: LP dual key over the slots that hold slack columns only -- keyed push tests,
# then the storm driver protocol.
set -u
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_vkey.py tests/test_gpu_lp.py > gpurun_out/r06j_tests.log 2>&1 || { tail -30 gpurun_out/r06j_tests.log; exit 1; }
tail -1 gpurun_out/r06j_tests.log
bash tools/ab_bench.sh r06j "" || exit 1
cat gpurun_out/r06j.txt

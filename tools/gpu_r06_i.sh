#!/bin/bash
# Round-6 GPU pass I: the pool build's FTRAN fast path (columns no eta pivot row touches) -- refresh
# parity tests (device == host build, single / two-pass FTRAN, sharded refresh, poison), then the
# storm driver protocol (pivots must be unchanged: 4.45).
set -u
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_pool_refresh.py tests/test_gpu_dist.py tests/test_gpu_poison.py tests/test_gpu_lp.py > gpurun_out/r06i_tests.log 2>&1 || { tail -30 gpurun_out/r06i_tests.log; exit 1; }
tail -1 gpurun_out/r06i_tests.log
bash tools/ab_bench.sh r06i "" || exit 1
cat gpurun_out/r06i.txt

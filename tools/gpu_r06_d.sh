#!/bin/bash
# Round-6 GPU pass D: LP parity tests, then the storm driver protocol and ssn (|V| = 16384) on this build.
set -u
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_lp.py tests/test_gpu_vkey.py tests/test_gpu_pool_refresh.py tests/test_gpu_kat.py tests/test_gpu_julia_mirror.py tests/test_gpu_sd_loop.py > gpurun_out/r06d_tests.log 2>&1 || { tail -30 gpurun_out/r06d_tests.log; exit 1; }
tail -2 gpurun_out/r06d_tests.log
bash tools/ab_bench.sh r06d "" "--instance ssn --scenarios 100000 --vertices 16384" || exit 1
cat gpurun_out/r06d.txt

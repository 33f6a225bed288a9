#!/bin/bash
# Round-5 GPU pass G: cut parity tests, the cut alone at 1M (fixup stamps variant, default
# build), a kernel trace of the bench protocol, then the driver's bench command.
set -u
mkdir -p gpurun_out
echo "cut tests"
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_cut.py tests/test_gpu_large_v.py tests/test_gpu_julia_mirror.py > gpurun_out/r05g_tests.log 2>&1 || { tail -30 gpurun_out/r05g_tests.log; exit 1; }
tail -2 gpurun_out/r05g_tests.log
echo "cut speed"
TWOSD_LIB=fxst TWOSD_FIX_STAMPS_PRINT=1 timeout -k 10 200 python3 -u tools/cut_speed.py 1000000 4096 3 || exit 1
timeout -k 10 200 python3 -u tools/cut_speed.py 1000000 4096 5 || exit 1
echo "trace"
bash tools/prof_trace.sh r05_tr3 || exit 1
echo "bench"
timeout -k 10 400 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r05g_bench.json 2> gpurun_out/r05g_bench.err || { tail -5 gpurun_out/r05g_bench.err; exit 1; }
tail -c 400 gpurun_out/r05g_bench.json

#!/bin/bash
# Round-5 GPU pass M: cut parity tests (with the truncate / push test), the storm cut alone, and
# the N = 8 per-rank emulation (after the fixup's small-batch grid change).
set -u
mkdir -p gpurun_out
echo "cut tests"
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_cut.py tests/test_gpu_large_v.py tests/test_gpu_julia_mirror.py tests/test_gpu_dist.py > gpurun_out/r05m_tests.log 2>&1 || { tail -30 gpurun_out/r05m_tests.log; exit 1; }
tail -2 gpurun_out/r05m_tests.log
echo "cut speed"
timeout -k 10 200 python3 -u tools/cut_speed.py 1000000 4096 5 || exit 1
timeout -k 10 200 python3 -u tools/cut_speed.py 125000 4096 5 || exit 1
echo "n8 emulation"
timeout -k 10 600 python3 -u tools/shard_emulate.py 8 1000000 20 2048 8192 5 > gpurun_out/r05m_n8.txt 2> gpurun_out/r05m_n8.err || { tail -5 gpurun_out/r05m_n8.err; exit 1; }
tail -1 gpurun_out/r05m_n8.txt

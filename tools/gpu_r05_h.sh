#!/bin/bash
# Round-5 GPU pass H: the whole GPU test suite and smoke(), the cut alone at 1M, then the N = 8
# per-rank emulation of the bench protocol (tools/shard_emulate.py, 2048-basis distributed pool).
set -u
mkdir -p gpurun_out profiles_tmp
echo "gpu tests"
timeout -k 10 900 python3 -u -m pytest --maxfail=5 -q --timeout 200 --timeout-method thread -m gpu tests > gpurun_out/r05h_tests.log 2>&1 || { tail -30 gpurun_out/r05h_tests.log; exit 1; }
tail -2 gpurun_out/r05h_tests.log
echo "smoke"
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05h_smoke.log 2>&1 || { tail -5 gpurun_out/r05h_smoke.log; exit 1; }
tail -1 gpurun_out/r05h_smoke.log
echo "cut speed"
timeout -k 10 200 python3 -u tools/cut_speed.py 1000000 4096 5 || exit 1
echo "n8 emulation"
timeout -k 10 600 python3 -u tools/shard_emulate.py 8 1000000 20 2048 8192 5 > gpurun_out/r05h_n8.txt 2> gpurun_out/r05h_n8.err || { tail -5 gpurun_out/r05h_n8.err; exit 1; }
tail -6 gpurun_out/r05h_n8.txt

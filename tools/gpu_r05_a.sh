#!/bin/bash
# Round-5 GPU session A: exact-tie cut tests, a traced bench (cut kernels), LP x_B unroll A/B and
# the refresh-pass A/B at x_EV.  Usage (GPU box, repo root): bash tools/gpu_r05_a.sh
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_cut.py tests/test_gpu_large_v.py > gpurun_out/r05_cut4.log 2>&1 || { tail -20 gpurun_out/r05_cut4.log; exit 1; }
tail -2 gpurun_out/r05_cut4.log
bash tools/prof_trace.sh r05_t2 --gpus 1 --steps 8 --warmup 4 --no-cpu --spot 4096 --trajectory 0 || exit 1
bash tools/ab_bench.sh r05_ab1 "" "TWOSD_LIB=xu2" "TWOSD_LIB=xu4" "--refresh-passes 2" || exit 1

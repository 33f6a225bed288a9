#!/bin/bash
# Round-5 GPU session B: cut tests after the row-batched fixup, then a traced bench.
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_cut.py tests/test_gpu_large_v.py tests/test_gpu_julia_mirror.py > gpurun_out/r05_cut6.log 2>&1 || { tail -30 gpurun_out/r05_cut5.log; exit 1; }
tail -2 gpurun_out/r05_cut6.log
bash tools/prof_trace.sh r05_t4 --gpus 1 --steps 8 --warmup 4 --no-cpu --spot 4096 --trajectory 0 || exit 1

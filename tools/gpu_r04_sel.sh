#!/bin/bash
# Round-4 sweep: two-level selection sizes (level-1 bases, candidates per level-1 pick) on the
# driver protocol; pivots vs selection time (one JSON line per setting)
mkdir -p gpurun_out/sel
A="--steps 20 --warmup 5 --no-cpu --spot 0 --trajectory 0"
bash tools/gpu_session.sh gpurun_out/sel \
  "c96|150|python bench.py $A --pool-cands 96 > gpurun_out/sel/c96.json" \
  "c128|150|python bench.py $A --pool-cands 128 > gpurun_out/sel/c128.json" \
  "c224|150|python bench.py $A --pool-cands 224 > gpurun_out/sel/c224.json" \
  "l64|150|python bench.py $A --pool-level1 64 > gpurun_out/sel/l64.json" \
  "l256|150|python bench.py $A --pool-level1 256 > gpurun_out/sel/l256.json" \
  "l64c224|150|python bench.py $A --pool-level1 64 --pool-cands 224 > gpurun_out/sel/l64c224.json"

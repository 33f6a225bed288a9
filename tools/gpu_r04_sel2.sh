#!/bin/bash
# Round-4 sweep, second pass: fewer level-1 groups with longer candidate lists
mkdir -p gpurun_out/sel2
A="--steps 20 --warmup 5 --no-cpu --spot 0 --trajectory 0"
bash tools/gpu_session.sh gpurun_out/sel2 \
  "l64c288|150|python bench.py $A --pool-level1 64 --pool-cands 288 > gpurun_out/sel2/l64c288.json" \
  "l32c224|150|python bench.py $A --pool-level1 32 --pool-cands 224 > gpurun_out/sel2/l32c224.json" \
  "l32c320|150|python bench.py $A --pool-level1 32 --pool-cands 320 > gpurun_out/sel2/l32c320.json" \
  "l48c256|150|python bench.py $A --pool-level1 48 --pool-cands 256 > gpurun_out/sel2/l48c256.json" \
  "l16c384|150|python bench.py $A --pool-level1 16 --pool-cands 384 > gpurun_out/sel2/l16c384.json" \
  "l64c224b|150|python bench.py $A --pool-level1 64 --pool-cands 224 > gpurun_out/sel2/l64c224b.json"

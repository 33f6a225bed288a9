#!/bin/bash
# Round-4 A/B: refresh pool size per x point (storm, driver protocol without extras)
A="--steps 20 --warmup 5 --no-cpu --spot 0 --trajectory 0"
bash tools/gpu_session.sh gpurun_out/s20 \
  "p4096|150|python bench.py $A > gpurun_out/s20/p4096.json" \
  "p6144|150|python bench.py $A --refresh-pool 6144 > gpurun_out/s20/p6144.json" \
  "p8192|150|python bench.py $A --refresh-pool 8192 > gpurun_out/s20/p8192.json" \
  "p8192t|150|python bench.py $A --refresh-pool 8192 --refresh-train 16384 > gpurun_out/s20/p8192t.json"

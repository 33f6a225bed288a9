#!/bin/bash
# Round-4 A/B: branch-free selection record step (selbf) against the default, storm driver protocol
A="--steps 20 --warmup 5 --no-cpu --spot 0 --trajectory 0"
bash tools/gpu_session.sh gpurun_out/s19 \
  "selbf|150|TWOSD_LIB=selbf python bench.py $A > gpurun_out/s19/storm_selbf.json" \
  "base|150|python bench.py $A > gpurun_out/s19/storm_base.json" \
  "selbf2|150|TWOSD_LIB=selbf python bench.py $A > gpurun_out/s19/storm_selbf2.json"

#!/bin/bash
# Round-4 sweep, third pass: the candidate settings on the trajectory (20 distinct SD candidates)
# and on ssn
mkdir -p gpurun_out/sel3
A="--steps 20 --warmup 5 --no-cpu --spot 0 --trajectory 20"
S="--instance ssn --scenarios 100000 --vertices 16384 --steps 8 --warmup 1 --no-cpu --spot 0 --trajectory 8"
bash tools/gpu_session.sh gpurun_out/sel3 \
  "d|150|python bench.py $A > gpurun_out/sel3/storm_l128c160.json" \
  "a|150|python bench.py $A --pool-level1 64 --pool-cands 224 > gpurun_out/sel3/storm_l64c224.json" \
  "b|150|python bench.py $A --pool-level1 16 --pool-cands 384 > gpurun_out/sel3/storm_l16c384.json" \
  "sd|200|python bench.py $S > gpurun_out/sel3/ssn_l128c160.json" \
  "sa|200|python bench.py $S --pool-level1 64 --pool-cands 224 > gpurun_out/sel3/ssn_l64c224.json"
bash tools/gpu_session.sh gpurun_out/sel3 \
  "ab_main|120|python tools/main_pivots.py" \
  "ab_eg3|120|TWOSD_LIB=eg3 python tools/main_pivots.py" \
  "ab_eg4|120|TWOSD_LIB=eg4 python tools/main_pivots.py"

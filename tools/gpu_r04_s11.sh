#!/bin/bash
# Round-4 A/B: eta-file traversal (BTRAN / FTRAN) -- group size 2 / 4 / 8, and the ping-pong
# prefetch of the next group (pp2 / pp4) -- on ssn (long eta files) and storm
S="--instance ssn --scenarios 100000 --vertices 16384 --steps 8 --warmup 1 --no-cpu --spot 0 --trajectory 0"
bash tools/gpu_session.sh gpurun_out/s11 \
  "ssn_base|200|python bench.py $S > gpurun_out/s11/ssn_base.json" \
  "ssn_eg4|200|TWOSD_LIB=eg4 python bench.py $S > gpurun_out/s11/ssn_eg4.json" \
  "ssn_eg8|200|TWOSD_LIB=eg8 python bench.py $S > gpurun_out/s11/ssn_eg8.json" \
  "ssn_pp2|200|TWOSD_LIB=pp2 python bench.py $S > gpurun_out/s11/ssn_pp2.json" \
  "ssn_pp4|200|TWOSD_LIB=pp4 python bench.py $S > gpurun_out/s11/ssn_pp4.json" \
  "st_base|120|python tools/main_pivots.py" \
  "st_eg8|120|TWOSD_LIB=eg8 python tools/main_pivots.py" \
  "st_pp2|120|TWOSD_LIB=pp2 python tools/main_pivots.py" \
  "st_pp4|120|TWOSD_LIB=pp4 python tools/main_pivots.py"

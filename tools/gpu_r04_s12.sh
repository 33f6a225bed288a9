#!/bin/bash
# Round-4 A/B: eta-group prefetch only for long eta files (pph) against the base and the
# always-prefetching build (pp2), ssn and storm
S="--instance ssn --scenarios 100000 --vertices 16384 --steps 8 --warmup 1 --no-cpu --spot 0 --trajectory 0"
A="--steps 20 --warmup 5 --no-cpu --spot 0 --trajectory 0"
bash tools/gpu_session.sh gpurun_out/s12 \
  "ssn_pph|200|TWOSD_LIB=pph python bench.py $S > gpurun_out/s12/ssn_pph.json" \
  "ssn_base|200|python bench.py $S > gpurun_out/s12/ssn_base.json" \
  "st_pph|120|TWOSD_LIB=pph python tools/main_pivots.py" \
  "st_base|120|python tools/main_pivots.py" \
  "st_pp2|120|TWOSD_LIB=pp2 python tools/main_pivots.py" \
  "bench_pph|150|TWOSD_LIB=pph python bench.py $A > gpurun_out/s12/storm_pph.json" \
  "bench_base|150|python bench.py $A > gpurun_out/s12/storm_base.json"

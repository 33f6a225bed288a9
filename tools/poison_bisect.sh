#!/bin/bash
# Which allocation family does the bench's LP path read before any kernel wrote it?  Runs the short
# bench with fresh allocations left as they come (none) and zero-filled by family (TWOSD_POISON=0,
# TWOSD_POISON_FAMILY bit 1 dalloc / 2 dgrow / 4 cut workspace), printing the per-step pivots.
# Zero fill only: a fill that yields wild indices can fault the GPU.
set -u
mkdir -p gpurun_out
for fam in ${FAMS:-none 7 1 2 4}; do
  if [ $fam = none ]; then E=""; else E="TWOSD_POISON=0 TWOSD_POISON_FAMILY=$fam"; fi
  env $E timeout -k 10 200 python3 bench.py --steps 8 --warmup 4 --no-cpu --spot 0 --trajectory 0 > gpurun_out/pb_$fam.json 2> gpurun_out/pb_$fam.err || { tail -3 gpurun_out/pb_$fam.err; exit 1; }
  python3 -c "
import json
d = json.loads(open('gpurun_out/pb_$fam.json').read().strip().splitlines()[-1])
print('$fam', [r[4] for r in d['steps_log']['rows']], d['lp_pivots_max'])"
done

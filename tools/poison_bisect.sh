#!/bin/bash
# Does any result of the bench depend on device memory no kernel wrote?  Runs the short bench with
# fresh allocations left as they come (none) and filled by family with BYTE (default 255: ints read
# back as -1, doubles as NaN; TWOSD_POISON_FAMILY bit 1 dalloc / 2 dgrow / 4 cut workspace),
# printing the per-step pivots and alpha.  The fill is synchronous (complete before the allocation
# returns), so it never races a kernel on the context's stream.  Stops at the first failing run.
set -u
mkdir -p gpurun_out
BYTE=${BYTE:-255}
for fam in ${FAMS:-none 7}; do
  if [ $fam = none ]; then E=""; else E="TWOSD_POISON=$BYTE TWOSD_POISON_FAMILY=$fam"; fi
  env $E timeout -k 10 240 python3 bench.py --steps 8 --warmup 4 --no-cpu --spot 0 --trajectory 0 > gpurun_out/pb_$fam.json 2> gpurun_out/pb_$fam.err || { tail -5 gpurun_out/pb_$fam.err; exit 1; }
  python3 -c "
import json
d = json.loads(open('gpurun_out/pb_$fam.json').read().strip().splitlines()[-1])
print('$fam', [r[4] for r in d['steps_log']['rows']], d['lp_pivots_max'], [p['alpha'] for p in d['x_points']])"
done

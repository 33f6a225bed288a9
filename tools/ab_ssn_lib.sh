#!/bin/bash
# A/B of LP-kernel variant libraries on the ssn 100k, |V| = 16384 config: bash tools/ab_ssn_lib.sh "v1 v2" [reps]
VARS=${1:-base}; REPS=${2:-2}
mkdir -p gpurun_out
for r in $(seq $REPS); do
  for v in $VARS; do
    TWOSD_LIB=$v timeout -k 10 300 python bench.py --instance ssn --scenarios 100000 --vertices 16384 --no-cpu --spot 0 --steps 4 --warmup 1 > gpurun_out/abssn_$v.log 2>> gpurun_out/abssn.err || exit 1
    python3 -c "
import json
d=json.loads(open('gpurun_out/abssn_$v.log').read().strip().splitlines()[-1])
print('$v', round(d['value']), round(d['ms_per_step'],2), 'lp', round(d['phases_ms_per_step']['lp_kernel'],2), 'piv', round(d['lp_pivots_mean'],3))
"
  done
done

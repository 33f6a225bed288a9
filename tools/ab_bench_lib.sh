#!/bin/bash
# A/B of LP-kernel variant libraries on the storm 1M bench step: bash tools/ab_bench_lib.sh "base v1 v2" [reps]
VARS=${1:-base}; REPS=${2:-2}
mkdir -p gpurun_out
: > gpurun_out/ablib.txt
for r in $(seq $REPS); do
  for v in $VARS; do
    TWOSD_LIB=$v timeout -k 10 300 python bench.py --no-cpu --spot 0 > gpurun_out/ablib_$v.log 2>> gpurun_out/ablib.err || exit 1
    python3 -c "
import json
d=json.loads(open('gpurun_out/ablib_$v.log').read().strip().splitlines()[-1])
print('$v', round(d['value']), round(d['ms_per_step'],2), 'lp', round(d['phases_ms_per_step']['lp_kernel'],2), 'piv', round(d['lp_pivots_mean'],3), 'refresh', [round(p['pool_refresh_ms'],1) for p in d['x_points']], [round(p['alpha'],4) for p in d['x_points']])
" | tee -a gpurun_out/ablib.txt
  done
done

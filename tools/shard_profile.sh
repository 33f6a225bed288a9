#!/bin/bash
# per-rank shard sizes of N = 2 / 4 / 8 on one GPU: step breakdown (no collectives)
mkdir -p gpurun_out
: > gpurun_out/shards.txt
for n in 125000 250000 500000; do
  timeout -k 10 300 python bench.py --no-cpu --spot 0 --scenarios $n > gpurun_out/shard_$n.log 2>> gpurun_out/shard.err || exit 1
  python3 -c "
import json
d=json.loads(open('gpurun_out/shard_$n.log').read().strip().splitlines()[-1])
print($n, round(d['ms_per_step'],2), {k:round(v,2) for k,v in d['phases_ms_per_step'].items()}, 'piv', round(d['lp_pivots_mean'],2), 'pool', d['config']['pool_refresh'])
for p in d['x_points']: print('   ', p['x'][:22], round(p['ms_per_step'],2), round(p['lp_kernel_ms'],2), round(p['lp_pivots_mean'],2), p['pool_refresh_parts_ms'])
" | tee -a gpurun_out/shards.txt
done

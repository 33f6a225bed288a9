#!/bin/bash
# pool size / two-level selection sweep at storm 1M (bench.py, no CPU baseline)
mkdir -p gpurun_out
: > gpurun_out/sweep2.jsonl
for a in "--pool 4096 --pool-cands 64" "--pool 6144 --pool-train 24576" "--pool 8192 --pool-train 32768" "--pool 8192 --pool-train 32768 --pool-level1 256" "--pool 12288 --pool-train 49152 --cand-train 131072"; do
  timeout -k 10 300 python bench.py --no-cpu --steps 3 --warmup 1 $a 2>>gpurun_out/sweep2.err | tail -1 | sed "s/^{/{\"args\": \"$a\", /" >> gpurun_out/sweep2.jsonl || exit 1
done
python3 -c "
import json
for l in open('gpurun_out/sweep2.jsonl'):
    d=json.loads(l); c=d['config']
    print(d['args'], '|', c['pool_build_s'], round(d['value']), round(d['ms_per_step'],2), round(d['lp_pivots_mean'],2), d['lp_pivots_max'], {k:round(v,2) for k,v in d['phases_ms_per_step'].items()})
"

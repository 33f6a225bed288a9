#!/bin/bash
# two-level selection sizes at pool 32768, storm 1M
mkdir -p gpurun_out
: > gpurun_out/sweep9.jsonl
run() { timeout -k 10 300 python bench.py --no-cpu --steps 3 --warmup 1 $1 2>>gpurun_out/sweep9.err | tail -1 | sed "s/^{/{\"args\": \"$1\", /" >> gpurun_out/sweep9.jsonl; }
run "--pool-level1 128 --pool-cands 192" || exit 1
run "--pool-level1 128 --pool-cands 224" || exit 1
run "--pool-level1 192 --pool-cands 160" || exit 1
run "--scenarios 125000 --pool-level1 128 --pool-cands 128" || exit 1
run "--scenarios 125000 --pool-level1 128 --pool-cands 160" || exit 1
python3 -c "
import json
for l in open('gpurun_out/sweep9.jsonl'):
    d=json.loads(l); c=d['config']
    print(d['args'], '|', c['pool_build_s'], round(d['value']), round(d['ms_per_step'],2), round(d['lp_pivots_mean'],3), {k:round(v,2) for k,v in d['phases_ms_per_step'].items()})
"

#!/bin/bash
# pool size beyond 16384 with a matching training set, storm 1M (step time incl. selection)
mkdir -p gpurun_out
: > gpurun_out/sweep6.jsonl
run() { timeout -k 10 300 python bench.py --no-cpu --steps 3 --warmup 1 $1 2>>gpurun_out/sweep6.err | tail -1 | sed "s/^{/{\"args\": \"$1\", /" >> gpurun_out/sweep6.jsonl; }
run "--pool 16384 --cand-train 262144" || exit 1
run "--pool 49152 --pool-train 196608 --cand-train 262144" || exit 1
run "--pool 65536 --pool-train 262144 --cand-train 524288" || exit 1
run "--pool 32768 --pool-train 131072 --cand-train 262144" || exit 1
python3 -c "
import json
for l in open('gpurun_out/sweep6.jsonl'):
    d=json.loads(l); c=d['config']
    print(d['args'], '|', c['pool_build_s'], round(d['value']), round(d['ms_per_step'],2), round(d['lp_pivots_mean'],3), {k:round(v,2) for k,v in d['phases_ms_per_step'].items()})
"

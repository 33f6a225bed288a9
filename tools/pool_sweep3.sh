#!/bin/bash
# larger pools at storm 1M and the 125k per-GPU share of 8 GPUs
mkdir -p gpurun_out
: > gpurun_out/sweep3.jsonl
run() { timeout -k 10 300 python bench.py --no-cpu --steps 3 --warmup 1 $1 2>>gpurun_out/sweep3.err | tail -1 | sed "s/^{/{\"args\": \"$1\", /" >> gpurun_out/sweep3.jsonl; }
run "--pool 16384 --pool-train 65536 --cand-train 131072" || exit 1
run "--pool 24576 --pool-train 98304 --cand-train 196608" || exit 1
run "--pool 32768 --pool-train 131072 --cand-train 262144" || exit 1
run "--scenarios 125000 --pool 4096" || exit 1
run "--scenarios 125000 --pool 12288 --pool-train 49152 --cand-train 131072" || exit 1
run "--scenarios 125000 --pool 24576 --pool-train 98304 --cand-train 196608" || exit 1
python3 -c "
import json
for l in open('gpurun_out/sweep3.jsonl'):
    d=json.loads(l); c=d['config']
    print(d['args'], '|', c['pool_build_s'], round(d['value']), round(d['ms_per_step'],2), round(d['lp_pivots_mean'],2), d['lp_pivots_max'], {k:round(v,2) for k,v in d['phases_ms_per_step'].items()})
"

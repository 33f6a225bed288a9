#!/bin/bash
# pool size vs per-GPU shard size (the N > 1 bench steps run 1M / N scenarios per rank)
mkdir -p gpurun_out
: > gpurun_out/sweep7.jsonl
run() { timeout -k 10 300 python bench.py --no-cpu --steps 5 --warmup 1 $1 2>>gpurun_out/sweep7.err | tail -1 | sed "s/^{/{\"args\": \"$1\", /" >> gpurun_out/sweep7.jsonl; }
for ns in 125000 250000 500000; do
  run "--scenarios $ns --pool 8192 --pool-train 32768 --cand-train 131072" || exit 1
  run "--scenarios $ns --pool 16384 --pool-train 65536 --cand-train 262144" || exit 1
  run "--scenarios $ns --pool 32768 --pool-train 131072 --cand-train 262144" || exit 1
done
python3 -c "
import json
for l in open('gpurun_out/sweep7.jsonl'):
    d=json.loads(l); c=d['config']
    print(d['args'], '|', c['pool_build_s'], round(d['value']), round(d['ms_per_step'],2), round(d['lp_pivots_mean'],3), {k:round(v,2) for k,v in d['phases_ms_per_step'].items()})
"

#!/bin/bash
# GPU tests + storm 1M bench at the flat and two-level pool configurations
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputests.log 2>&1 || { tail -30 gpurun_out/gputests.log; exit 1; }
tail -2 gpurun_out/gputests.log
: > gpurun_out/cur.jsonl
for a in "--pool 512" "--pool 4096 --pool-level1 128 --pool-cands 128"; do
  TWOSD_DEBUG=1 timeout -k 10 300 python bench.py --no-cpu --steps 3 --warmup 1 $a 2>>gpurun_out/cur.err | tail -1 >> gpurun_out/cur.jsonl || exit 1
done
python3 -c "
import json
for l in open('gpurun_out/cur.jsonl'):
    d=json.loads(l); c=d['config']
    print(c['basis_pool'], c['pool_selection'], c['pool_build_s'], round(d['value']), round(d['ms_per_step'],2), round(d['lp_pivots_mean'],2), {k:round(v,2) for k,v in d['phases_ms_per_step'].items()})
"
grep prepare_x gpurun_out/cur.err | sort | uniq -c | head -20

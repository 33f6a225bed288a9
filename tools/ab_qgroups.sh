#!/bin/bash
# A/B of the XCD-grouped LP work queues (TWOSD_QGROUPS=1: one global queue) at storm 1M and 125k
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_lp.py -x -q --timeout 120 --timeout-method thread > gpurun_out/gputests.log 2>&1 || { tail -30 gpurun_out/gputests.log; exit 1; }
tail -1 gpurun_out/gputests.log
: > gpurun_out/ab.jsonl
for ns in 1000000 125000; do
for q in 1 8; do
  TWOSD_QGROUPS=$q timeout -k 10 300 python bench.py --no-cpu --steps 3 --warmup 1 --scenarios $ns --pool 4096 --pool-level1 128 --pool-cands 128 2>>gpurun_out/ab.err | tail -1 | sed "s/^{/{\"q\": $q, /" >> gpurun_out/ab.jsonl || exit 1
done
done
python3 -c "
import json
for l in open('gpurun_out/ab.jsonl'):
    d=json.loads(l); c=d['config']
    print('q',d['q'], c['scenarios'], round(d['value']), round(d['ms_per_step'],2), round(d['lp_pivots_mean'],2), {k:round(v,2) for k,v in d['phases_ms_per_step'].items()})
"

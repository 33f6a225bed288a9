#!/bin/bash
# queue-group count sweep (TWOSD_QGROUPS) at storm 1M and 125k, bench defaults
mkdir -p gpurun_out
: > gpurun_out/qg.jsonl
for ns in 125000 1000000; do
for q in 8 16 32 64; do
  TWOSD_QGROUPS=$q timeout -k 10 300 python bench.py --no-cpu --steps 3 --warmup 1 --scenarios $ns 2>>gpurun_out/qg.err | tail -1 | sed "s/^{/{\"q\": $q, /" >> gpurun_out/qg.jsonl || exit 1
done
done
python3 -c "
import json
for l in open('gpurun_out/qg.jsonl'):
    d=json.loads(l); c=d['config']
    print('q',d['q'], c['scenarios'], round(d['value']), round(d['ms_per_step'],2), {k:round(v,2) for k,v in d['phases_ms_per_step'].items()})
"

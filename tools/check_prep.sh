#!/bin/bash
# GPU tests + storm bench (1M, 125k) with the device-built selection stream
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputests.log 2>&1 || { tail -30 gpurun_out/gputests.log; exit 1; }
tail -1 gpurun_out/gputests.log
: > gpurun_out/prep.jsonl
: > gpurun_out/prep.err
for ns in 1000000 125000; do
  TWOSD_DEBUG=1 timeout -k 10 300 python bench.py --no-cpu --steps 3 --warmup 1 --scenarios $ns --pool 4096 --pool-level1 128 --pool-cands 128 2>>gpurun_out/prep.err | tail -1 >> gpurun_out/prep.jsonl || exit 1
done
python3 -c "
import json
for l in open('gpurun_out/prep.jsonl'):
    d=json.loads(l); c=d['config']
    print(c['scenarios'], round(d['value']), round(d['ms_per_step'],2), d['lp_pivots_mean'], d['alpha_check'], {k:round(v,2) for k,v in d['phases_ms_per_step'].items()})
"
grep prepare_x gpurun_out/prep.err | tail -8

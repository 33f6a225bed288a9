#!/bin/bash
# A/B of the hardest-first LP visiting order (TWOSD_LPT_FRAC) at storm 1M and 125k
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_lp.py -x -q --timeout 120 --timeout-method thread > gpurun_out/gputests.log 2>&1 || { tail -30 gpurun_out/gputests.log; exit 1; }
tail -1 gpurun_out/gputests.log
: > gpurun_out/lpt.jsonl
for ns in 1000000 125000; do
for f in 0 0.05 0.02; do
  TWOSD_LPT_FRAC=$f timeout -k 10 300 python bench.py --no-cpu --steps 3 --warmup 1 --scenarios $ns 2>>gpurun_out/lpt.err | tail -1 | sed "s/^{/{\"f\": $f, /" >> gpurun_out/lpt.jsonl || exit 1
done
done
python3 -c "
import json
for l in open('gpurun_out/lpt.jsonl'):
    d=json.loads(l); c=d['config']
    print('lpt',d['f'], c['scenarios'], round(d['value']), round(d['ms_per_step'],2), round(d['lp_pivots_mean'],3), {k:round(v,2) for k,v in d['phases_ms_per_step'].items()})
"

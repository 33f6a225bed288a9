#!/bin/bash
# A/B of LP kernel builds (tools/build_variants.sh) through bench.py defaults: bash tools/ab_bench.sh "v1 v2 ..." [scenarios]
VARS=${1:-base}
NS=${2:-1000000}
mkdir -p gpurun_out
: > gpurun_out/abb.jsonl
for v in $VARS; do
  if [ "$v" = default ]; then unset TWOSD_LIB; else export TWOSD_LIB=$v; fi
  timeout -k 10 300 python bench.py --no-cpu --steps 3 --warmup 1 --scenarios $NS 2>>gpurun_out/abb.err | tail -1 | sed "s/^{/{\"lib\": \"$v\", /" >> gpurun_out/abb.jsonl || exit 1
done
python3 -c "
import json
for l in open('gpurun_out/abb.jsonl'):
    d=json.loads(l)
    print(d['lib'], round(d['value']), round(d['ms_per_step'],2), round(d['lp_pivots_mean'],3), d['alpha_check'], {k:round(v,2) for k,v in d['phases_ms_per_step'].items()})
"

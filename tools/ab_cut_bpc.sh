#!/bin/bash
# cut_argmax grid: 3 blocks per CU (old) vs resident occupancy (default), storm 1M and 125k
mkdir -p gpurun_out
: > gpurun_out/cutbpc.jsonl
run() { env $1 timeout -k 10 300 python bench.py --no-cpu --steps 5 --warmup 1 $2 2>>gpurun_out/cutbpc.err | tail -1 | sed "s/^{/{\"args\": \"$1 $2\", /" >> gpurun_out/cutbpc.jsonl; }
run TWOSD_CUT_BPC=3 "" || exit 1
run TWOSD_CUT_BPC=0 "" || exit 1
run TWOSD_CUT_BPC=3 "--scenarios 125000" || exit 1
run TWOSD_CUT_BPC=0 "--scenarios 125000" || exit 1
python3 -c "
import json
for l in open('gpurun_out/cutbpc.jsonl'):
    d=json.loads(l)
    print(d['args'], '|', round(d['value']), round(d['ms_per_step'],2), repr(d['alpha_check']), round(d['cutgen']['t_ms'],3), round(d['cutgen']['frac_measured'],3))
"

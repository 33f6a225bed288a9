#!/bin/bash
# N=1 bench and an N=2 rehearsal of the multi-rank bench path (both ranks on cuda:0, gloo)
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --no-cpu --steps 2 --warmup 1 > gpurun_out/n1.json 2> gpurun_out/n1.err || { tail -20 gpurun_out/n1.err; exit 1; }
TWOSD_BENCH_SHARED_GPU=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --steps 2 --warmup 1 --no-cpu > gpurun_out/n2.json 2> gpurun_out/n2.err || { tail -20 gpurun_out/n2.err; exit 1; }
python3 -c "
import json
for f in ['gpurun_out/n1.json','gpurun_out/n2.json']:
    d=json.loads(open(f).read().strip().splitlines()[-1])
    print(f, d['n_gpus'], round(d['value']), round(d['ms_per_step'],2), repr(d['alpha_check']), d['config']['workload'], {k:round(v,2) for k,v in d['phases_ms_per_step'].items()})
"

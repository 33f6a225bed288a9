#!/bin/bash
# N=1 bench and an N=2 rehearsal of the multi-rank bench path (both ranks on cuda:0, gloo):
# same scenarios and x points, so the per-x cut alphas must agree (exact histogram, rank-ordered sums)
NS=${1:-200000}
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --scenarios $NS --no-cpu --spot 0 --steps 4 --warmup 1 > gpurun_out/n1.json 2> gpurun_out/n1.err || { tail -20 gpurun_out/n1.err; exit 1; }
TWOSD_BENCH_SHARED_GPU=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --scenarios $NS --gpus 2 --steps 4 --warmup 1 --no-cpu --spot 0 > gpurun_out/n2.json 2> gpurun_out/n2.err || { tail -20 gpurun_out/n2.err; exit 1; }
python3 -c "
import json
ds=[json.loads(open(f).read().strip().splitlines()[-1]) for f in ['gpurun_out/n1.json','gpurun_out/n2.json']]
for d in ds:
    print(d['n_gpus'], round(d['value']), round(d['ms_per_step'],2), d['config']['workload'], {k:round(v,2) for k,v in d['phases_ms_per_step'].items()})
for a, b in zip(ds[0]['x_points'], ds[1]['x_points']):
    print(a['x'], repr(a['alpha']), repr(b['alpha']), abs(a['alpha'] - b['alpha']) / abs(a['alpha']))
"

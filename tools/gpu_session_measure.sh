#!/bin/bash
# Measurement session (GPU box, repo root): the driver's bench command line, the other BASELINE
# configs, and the N = 8 per-rank step emulated on one GPU.  Every GPU step has its own limit and
# the script stops at the first failure.
set -u
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/driver_bench.json 2> gpurun_out/driver_bench.err || { echo "driver bench failed"; tail -5 gpurun_out/driver_bench.err; exit 1; }
python3 -c "
import json; d = json.loads(open('gpurun_out/driver_bench.json').read().strip().splitlines()[-1])
print('driver bench', round(d['value'] / 1e6, 3), 'M/s', round(d['ms_per_step'], 2), 'ms', {k: round(v, 2) for k, v in d['phases_ms_per_step'].items()})"
bash tools/configs_r03.sh || exit 1
for P in 1024 4096; do
  timeout -k 10 400 python tools/shard_emulate.py 8 1000000 8 $P > gpurun_out/shard_emulate_pool$P.txt 2>&1 || { echo "shard emulate $P failed"; tail -5 gpurun_out/shard_emulate_pool$P.txt; exit 1; }
  tail -1 gpurun_out/shard_emulate_pool$P.txt
done

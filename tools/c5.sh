set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_lp.py -x -q --timeout 120 --timeout-method thread > gpurun_out/gputests.log 2>&1
tail -2 gpurun_out/gputests.log
: > gpurun_out/c5.jsonl
for a in "--pool 4096 --pool-level1 256 --pool-cands 128" "--pool 4096 --pool-level1 128 --pool-cands 128" "--pool 6144 --pool-train 24576 --pool-level1 256 --pool-cands 128"; do
  timeout -k 10 300 python bench.py --no-cpu --steps 3 --warmup 1 $a 2>>gpurun_out/c5.err | tail -1 >> gpurun_out/c5.jsonl
done
python3 -c "
import json
for l in open('gpurun_out/c5.jsonl'):
    d=json.loads(l); c=d['config']; print(c['basis_pool'], c['pool_selection'], c['pool_build_s'], round(d['value']), round(d['ms_per_step'],2), round(d['lp_pivots_mean'],2), {k:round(v,2) for k,v in d['phases_ms_per_step'].items()})
"

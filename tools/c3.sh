set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_lp.py -x -q --timeout 120 --timeout-method thread > gpurun_out/gputests.log 2>&1
tail -2 gpurun_out/gputests.log
: > gpurun_out/c3.jsonl
for a in "--pool 512" "--pool 1024" "--pool 2048"; do
  timeout -k 10 300 python bench.py --no-cpu --steps 3 --warmup 1 $a 2>/dev/null | tail -1 >> gpurun_out/c3.jsonl
done
python3 -c "
import json
for l in open('gpurun_out/c3.jsonl'):
    d=json.loads(l); print(d['config']['scenarios'], d['config']['basis_pool'], round(d['value']), round(d['ms_per_step'],2), round(d['lp_pivots_mean'],2), {k:round(v,2) for k,v in d['phases_ms_per_step'].items()})
"

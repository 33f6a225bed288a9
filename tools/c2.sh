set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputests.log 2>&1
tail -2 gpurun_out/gputests.log
: > gpurun_out/c2.jsonl
for a in "" "--scenarios 125000"; do
  timeout -k 10 300 python bench.py --no-cpu --steps 5 --warmup 1 $a 2>/dev/null | tail -1 >> gpurun_out/c2.jsonl
done
python3 -c "
import json
for l in open('gpurun_out/c2.jsonl'):
    d=json.loads(l); print(d['config']['scenarios'], d['config']['vertices'], round(d['value']), round(d['ms_per_step'],2), {k:round(v,2) for k,v in d['phases_ms_per_step'].items()})
"

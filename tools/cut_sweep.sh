# cut kernel |V| sweep (storm 1M, no CPU leg): bash tools/cut_sweep.sh -> gpurun_out/cut_sweep.jsonl
set -e
mkdir -p gpurun_out
: > gpurun_out/cut_sweep.jsonl
for v in ${VS:-64 512 4096}; do
  timeout -k 10 300 python bench.py --no-cpu --steps 3 --warmup 1 --vertices $v 2>> gpurun_out/cut_sweep.err | tail -1 >> gpurun_out/cut_sweep.jsonl
done
python3 - <<'PY'
import json
for l in open('gpurun_out/cut_sweep.jsonl'):
    d = json.loads(l); c = d['cutgen']
    print(d['config']['vertices'], 'cut_ms', round(c['t_ms'], 3), 'GB/s', round(c['hbm_gbs'], 1), 'TF', round(c.get('mfma_tflops', 0), 1), 'frac', round(c['frac'], 3), 'value', round(d['value']))
PY

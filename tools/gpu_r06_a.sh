#!/bin/bash
# Round-6 GPU pass A: the GPU suite + smoke, the ssn |V| = 16384 config with the old 256-pivot
# eta file (TWOSD_KMAX=256) and the LDS-sized default, and the driver's bench command.
set -u
mkdir -p gpurun_out
bash tools/gpu_r06_tests.sh r06a || exit 1
for K in 256 default; do
  if [ $K = default ]; then E=""; else E="TWOSD_KMAX=$K"; fi
  env $E timeout -k 10 300 python3 bench.py --instance ssn --scenarios 100000 --vertices 16384 --spot 1024 --no-cpu --steps 8 --warmup 1 --trajectory 0 > gpurun_out/r06a_ssn_$K.json 2> gpurun_out/r06a_ssn_$K.err || { tail -5 gpurun_out/r06a_ssn_$K.err; exit 1; }
  python3 -c "
import json
d = json.loads(open('gpurun_out/r06a_ssn_$K.json').read().strip().splitlines()[-1])
print('ssn kmax $K', round(d['ms_per_step'], 2), 'ms', d['phases_ms_per_step'], 'pivots', round(d['lp_pivots_mean'], 2), d['lp_pivots_max'], 'retries', d['lp_iter_limit_retries'], [round(x['alpha_rel_err'], 18) for x in d['parity_spot_check']])"
done
timeout -k 10 400 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r06a_bench.json 2> gpurun_out/r06a_bench.err || { tail -5 gpurun_out/r06a_bench.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/r06a_bench.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['phases_ms_per_step'], d['lp_pivots_mean'], d['lp_iter_limit_retries'], d['cutgen']['frac'], [ (x['alpha_rel_err'], x['beta_max_rel_err']) for x in d['parity_spot_check']], d['cpu_baseline']['value'])"

#!/bin/bash
# Round-5 final GPU check: the whole GPU suite, smoke(), and the driver's bench command.
set -u
mkdir -p gpurun_out
echo "gpu tests"
timeout -k 10 900 python3 -u -m pytest --maxfail=5 -q --timeout 200 --timeout-method thread -m gpu tests > gpurun_out/r05z_tests.log 2>&1 || { tail -30 gpurun_out/r05z_tests.log; exit 1; }
tail -2 gpurun_out/r05z_tests.log
echo "smoke"
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05z_smoke.log 2>&1 || { tail -5 gpurun_out/r05z_smoke.log; exit 1; }
tail -1 gpurun_out/r05z_smoke.log
echo "bench"
timeout -k 10 400 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r05z_bench.json 2> gpurun_out/r05z_bench.err || { tail -5 gpurun_out/r05z_bench.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/r05z_bench.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['phases_ms_per_step'], d['cutgen']['frac'], [ (x['alpha_rel_err'], x['beta_max_rel_err']) for x in d['parity_spot_check']])"

#!/bin/bash
# Round-5 GPU pass Q: cut parity tests, the storm cut alone, the driver's bench command and the
# other configs (after the band moved to the scalar cache and the log addresses to the log path).
set -u
mkdir -p gpurun_out
echo "cut tests"
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_cut.py tests/test_gpu_large_v.py tests/test_gpu_julia_mirror.py > gpurun_out/r05q_tests.log 2>&1 || { tail -30 gpurun_out/r05q_tests.log; exit 1; }
tail -2 gpurun_out/r05q_tests.log
echo "cut speed"
timeout -k 10 200 python3 -u tools/cut_speed.py 1000000 4096 5 || exit 1
echo "bench"
timeout -k 10 400 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r05q_bench.json 2> gpurun_out/r05q_bench.err || { tail -5 gpurun_out/r05q_bench.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/r05q_bench.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['phases_ms_per_step'], d['cutgen']['frac'], [ (x['alpha_rel_err'], x['beta_max_rel_err']) for x in d['parity_spot_check']])"
echo "configs"
bash tools/configs_r05.sh

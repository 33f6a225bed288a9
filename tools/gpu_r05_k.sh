#!/bin/bash
# Round-5 GPU pass K: the whole GPU suite, the storm cut alone, the driver's bench command and the
# other BASELINE configs (after the PK / twin-index maintenance change).
set -u
mkdir -p gpurun_out
echo "gpu tests"
timeout -k 10 900 python3 -u -m pytest --maxfail=5 -q --timeout 200 --timeout-method thread -m gpu tests > gpurun_out/r05k_tests.log 2>&1 || { tail -30 gpurun_out/r05k_tests.log; exit 1; }
tail -2 gpurun_out/r05k_tests.log
echo "cut speed"
timeout -k 10 200 python3 -u tools/cut_speed.py 1000000 4096 5 || exit 1
echo "bench"
timeout -k 10 400 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r05k_bench.json 2> gpurun_out/r05k_bench.err || { tail -5 gpurun_out/r05k_bench.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/r05k_bench.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['phases_ms_per_step'], d['cutgen']['frac'])"
echo "configs"
bash tools/configs_r05.sh

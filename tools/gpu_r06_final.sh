#!/bin/bash
# Round-6 final evidence on the final build: the whole GPU suite + smoke() (tools/gpu_r06_tests.sh),
# then the driver's bench command line, its JSON line kept as gpurun_out/r06final_bench.json.
set -u
mkdir -p gpurun_out
bash tools/gpu_r06_tests.sh r06final || exit 1
timeout -k 10 900 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r06final_bench.json 2> gpurun_out/r06final_bench.err || { tail -20 gpurun_out/r06final_bench.err; exit 1; }
tail -c 600 gpurun_out/r06final_bench.json

#!/bin/bash
# Round-5 GPU pass C: the cut parity tests, the driver's bench command, the poison check (zero fill of every
# allocation family vs none) and the ssn warm-start hindsight table (tools/ssn_hindsight.py).
set -u
mkdir -p gpurun_out
echo "cut tests"
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_cut.py tests/test_gpu_large_v.py tests/test_gpu_julia_mirror.py > gpurun_out/r05c_tests.log 2>&1 || { tail -30 gpurun_out/r05c_tests.log; exit 1; }
tail -2 gpurun_out/r05c_tests.log
echo "bench"
timeout -k 10 400 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r05c_bench.json 2> gpurun_out/r05c_bench.err || { tail -5 gpurun_out/r05c_bench.err; exit 1; }
tail -c 600 gpurun_out/r05c_bench.json
echo "poison"
FAMS="none 7" bash tools/poison_bisect.sh || exit 1
echo "ssn hindsight"
timeout -k 10 400 python3 -u tools/ssn_hindsight.py 500 16 > gpurun_out/r05c_ssn_hindsight.txt 2> gpurun_out/r05c_ssn.err || { tail -5 gpurun_out/r05c_ssn.err; exit 1; }
cat gpurun_out/r05c_ssn_hindsight.txt

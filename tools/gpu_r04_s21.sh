#!/bin/bash
# Round-4: one FTRAN pass in the pool build (pg_gather_kernel) -- parity tests, then the storm A/B
A="--steps 20 --warmup 5 --no-cpu --spot 0 --trajectory 0"
T="python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu"
bash tools/gpu_session.sh gpurun_out/s21 \
  "tests|300|$T tests/test_gpu_pool_refresh.py tests/test_gpu_dist.py" \
  "gather|150|python bench.py $A > gpurun_out/s21/gather.json" \
  "twopass|150|TWOSD_PG_NOSCRATCH=1 python bench.py $A > gpurun_out/s21/twopass.json" \
  "gather2|150|python bench.py $A > gpurun_out/s21/gather2.json"

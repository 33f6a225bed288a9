#!/bin/bash
# Round-4: pool fill walks with 4 columns in flight -- parity tests, then storm benches
A="--steps 20 --warmup 5 --no-cpu --spot 0 --trajectory 0"
T="python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu"
bash tools/gpu_session.sh gpurun_out/s22 \
  "tests|300|$T tests/test_gpu_pool_refresh.py tests/test_gpu_dist.py" \
  "fill4|150|python bench.py $A > gpurun_out/s22/fill4.json" \
  "fill4b|150|python bench.py $A > gpurun_out/s22/fill4b.json" \
  "trace|200|rocprofv3 --kernel-trace --stats -d gpurun_out/s22/prof -o run -- python bench.py $A > gpurun_out/s22/trace_bench.json && python tools/prof_reduce.py gpurun_out/s22/prof gpurun_out/s22/trace"

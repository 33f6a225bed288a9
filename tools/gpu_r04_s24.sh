#!/bin/bash
# Round-4: per-wave dual-set keys, block-reduced LP stats, candidate lists built during the level-1
# pass, LDS-staged gather -- full GPU tests, then storm benches and a kernel + HIP API trace
A="--steps 20 --warmup 5 --no-cpu --spot 0 --trajectory 0"
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu"
bash tools/gpu_session.sh gpurun_out/s24 \
  "tests|600|$T tests" \
  "b1|150|python bench.py $A > gpurun_out/s24/b1.json" \
  "b2|150|python bench.py $A > gpurun_out/s24/b2.json" \
  "api|300|cd /tmp && rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv -d \$GRAFT_REPO_ROOT/gpurun_out/s24/prof -o run -- python3 \$GRAFT_REPO_ROOT/bench.py --steps 8 --warmup 5 --no-cpu --spot 0 --trajectory 0 > \$GRAFT_REPO_ROOT/gpurun_out/s24/api_bench.json && cd \$GRAFT_REPO_ROOT && for f in \$(find gpurun_out/s24/prof -name '*trace.csv'); do gzip -c \$f > gpurun_out/s24/\$(basename \$f).gz; done && rm -rf gpurun_out/s24/prof"

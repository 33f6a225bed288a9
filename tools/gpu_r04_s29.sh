#!/bin/bash
# Round-4: the refresh's training solves on a kernel variant without the vertex recovery (MODE 1)
A="--steps 20 --warmup 5 --no-cpu --spot 0 --trajectory 0"
bash tools/gpu_session.sh gpurun_out/s29 \
  "tests|300|python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "b1|150|python bench.py $A > gpurun_out/s29/b1.json" \
  "b2|150|python bench.py $A > gpurun_out/s29/b2.json" \
  "trace|200|cd /tmp && rocprofv3 --kernel-trace --stats --output-format csv -d \$GRAFT_REPO_ROOT/gpurun_out/s29/prof -o run -- python3 \$GRAFT_REPO_ROOT/bench.py $A > \$GRAFT_REPO_ROOT/gpurun_out/s29/trace_bench.json && cd \$GRAFT_REPO_ROOT && python3 tools/prof_reduce.py gpurun_out/s29/prof gpurun_out/s29/trace"

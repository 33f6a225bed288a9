#!/bin/bash
# Round-4 closing check after the cut occupancy change: GPU tests, smoke, the storm bench line, configs
bash tools/gpu_session.sh gpurun_out/final4 \
  "tests|300|python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "smoke|120|python -c 'import __graft_entry__ as g; g.smoke()'" \
  "bench|300|python bench.py --steps 20 --warmup 5 > gpurun_out/final4/bench.json" \
  "configs|600|bash tools/configs_r04.sh"

#!/bin/bash
# Round-4 last check of the shipped tree: GPU tests, smoke, the driver's bench line
bash tools/gpu_session.sh gpurun_out/final5 \
  "tests|300|python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread" \
  "smoke|120|python -c 'import __graft_entry__ as g; g.smoke()'" \
  "bench|300|python bench.py --steps 20 --warmup 5 > gpurun_out/final5/bench.json"

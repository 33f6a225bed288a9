#!/bin/bash
# Round-4 session: GPU tests, main-pivot LP timing and the driver-protocol bench of the current library
bash tools/gpu_session.sh gpurun_out/s8 \
  "tests|300|python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "ab_main|120|python tools/main_pivots.py" \
  "bench|300|python bench.py --steps 20 --warmup 5 > gpurun_out/s8/bench.json"

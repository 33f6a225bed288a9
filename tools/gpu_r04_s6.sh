#!/bin/bash
# Round-4 session: GPU tests and bench of the current library, then the profile passes
bash tools/gpu_session.sh gpurun_out/s6 \
  "tests|300|python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "bench|300|python bench.py > gpurun_out/s6/bench.json" \
  "ab_main|120|python tools/main_pivots.py" \
  "profile|780|bash tools/profile_r04.sh r04"

#!/bin/bash
# Round-4 closing session: GPU tests and smoke on the final tree, the driver's command under
# rocprofv3 (trace + PMC passes), then the full bench line
bash tools/gpu_session.sh gpurun_out/final2 \
  "tests|300|python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "smoke|120|python -c 'import __graft_entry__ as g; g.smoke()'" \
  "profile|700|bash tools/profile_r04.sh r04b" \
  "bench|300|python bench.py --steps 20 --warmup 5 > gpurun_out/final2/bench.json"

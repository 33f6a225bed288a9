#!/bin/bash
# Round-4 closing session (third): GPU tests and smoke on the final tree, the driver's command
# under rocprofv3 (trace + PMC passes), the full bench line, the N = 8 emulation at the bench's pool
bash tools/gpu_session.sh gpurun_out/final3 \
  "tests|300|python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "smoke|120|python -c 'import __graft_entry__ as g; g.smoke()'" \
  "profile|700|bash tools/profile_r04.sh r04c" \
  "bench|300|python bench.py --steps 20 --warmup 5 > gpurun_out/final3/bench.json" \
  "n8|400|python tools/shard_emulate.py 8 1000000 20 2048 8192 5 > gpurun_out/final3/shard_emulate_pool2048.txt"

#!/bin/bash
# Round-4 final measurement session: the driver's command under rocprofv3 (trace + PMC passes,
# reduced on the box), the full bench line (CPU baseline, spot checks, trajectory), and the
# other BASELINE configs
bash tools/gpu_session.sh gpurun_out/final \
  "profile|700|bash tools/profile_r04.sh r04" \
  "bench|300|python bench.py --steps 20 --warmup 5 > gpurun_out/final/bench.json" \
  "configs|600|bash tools/configs_r04.sh"

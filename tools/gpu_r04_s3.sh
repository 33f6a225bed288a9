#!/bin/bash
# Round-4 session: N = 8 per-rank step emulated on one GPU (distributed refresh pools 1024 / 2048),
# then the BASELINE configs
bash tools/gpu_session.sh gpurun_out/s4 \
  "emu1024|330|python -u tools/shard_emulate.py 8 1000000 8 1024 > gpurun_out/s4/shard_emulate_pool1024.txt" \
  "emu2048|330|python -u tools/shard_emulate.py 8 1000000 8 2048 > gpurun_out/s4/shard_emulate_pool2048.txt" \
  "configs|500|bash tools/configs_r04.sh"

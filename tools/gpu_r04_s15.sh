#!/bin/bash
# Round-4 session: N = 8 per-rank step emulated on one GPU with the bench warmup, pool sizes
# 1024 / 1536 / 3072 (2048 / 4096: gpu_r04_s14.sh)
bash tools/gpu_session.sh gpurun_out/s15 \
  "emu1024|500|python -u tools/shard_emulate.py 8 1000000 20 1024 4096 5 > gpurun_out/s15/shard_emulate_pool1024.txt" \
  "emu1536|500|python -u tools/shard_emulate.py 8 1000000 20 1536 6144 5 > gpurun_out/s15/shard_emulate_pool1536.txt" \
  "emu3072|500|python -u tools/shard_emulate.py 8 1000000 20 3072 12288 5 > gpurun_out/s15/shard_emulate_pool3072.txt"

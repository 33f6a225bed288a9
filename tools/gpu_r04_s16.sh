#!/bin/bash
# Round-4 session: selection chunks up to 64 per tile (small batches) -- GPU tests, then the N = 8
# emulation at pools 2048 / 4096 and the storm bench
bash tools/gpu_session.sh gpurun_out/s16 \
  "tests|300|python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "emu2048|500|python -u tools/shard_emulate.py 8 1000000 20 2048 8192 5 > gpurun_out/s16/shard_emulate_pool2048.txt" \
  "emu4096|500|python -u tools/shard_emulate.py 8 1000000 20 4096 16384 5 > gpurun_out/s16/shard_emulate_pool4096.txt" \
  "storm|150|python bench.py --steps 20 --warmup 5 --no-cpu --spot 0 --trajectory 0 > gpurun_out/s16/storm.json"

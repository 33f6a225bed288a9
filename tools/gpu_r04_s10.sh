#!/bin/bash
# Round-4 session: LP phase shares (stamps build) on storm and ssn, then the N = 8 per-rank step
# emulated on one GPU (pool 2048 / 4096)
bash tools/gpu_session.sh gpurun_out/s10 \
  "phases_storm|200|TWOSD_LIB=stamps python tools/lp_phases_bench.py 250000 4096 16384 storm" \
  "phases_ssn|200|TWOSD_LIB=stamps python tools/lp_phases_bench.py 100000 512 2048 ssn" \
  "emu4096|400|python -u tools/shard_emulate.py 8 1000000 8 4096 > gpurun_out/s10/shard_emulate_pool4096.txt" \
  "emu2048|400|python -u tools/shard_emulate.py 8 1000000 8 2048 > gpurun_out/s10/shard_emulate_pool2048.txt"

#!/bin/bash
# Round-4 session: row-broadcast wave reductions -- GPU tests, storm and ssn, then the N = 8
# per-rank step emulated with the bench's warmup (pool 4096 and 2048)
S="--instance ssn --scenarios 100000 --vertices 16384 --steps 8 --warmup 1 --no-cpu --spot 0 --trajectory 0"
A="--steps 20 --warmup 5 --no-cpu --spot 0 --trajectory 0"
bash tools/gpu_session.sh gpurun_out/s14 \
  "tests|300|python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "storm|150|python bench.py $A > gpurun_out/s14/storm.json" \
  "ssn|200|python bench.py $S > gpurun_out/s14/ssn.json" \
  "emu4096|500|python -u tools/shard_emulate.py 8 1000000 20 4096 16384 5 > gpurun_out/s14/shard_emulate_pool4096.txt" \
  "emu2048|500|python -u tools/shard_emulate.py 8 1000000 20 2048 8192 5 > gpurun_out/s14/shard_emulate_pool2048.txt"

#!/bin/bash
# Round-4 session: DPP moves without a preset old value -- GPU tests, storm and ssn
S="--instance ssn --scenarios 100000 --vertices 16384 --steps 8 --warmup 1 --no-cpu --spot 0 --trajectory 0"
A="--steps 20 --warmup 5 --no-cpu --spot 0 --trajectory 0"
bash tools/gpu_session.sh gpurun_out/s18 \
  "tests|300|python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "storm|150|python bench.py $A > gpurun_out/s18/storm.json" \
  "ssn|200|python bench.py $S > gpurun_out/s18/ssn.json" \
  "ab_main|120|python tools/main_pivots.py"

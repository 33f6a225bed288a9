#!/bin/bash
# Round-4 session: long-solves-first visiting order -- GPU tests, then storm and ssn with and
# without it (TWOSD_LONG_FIRST=0)
A="--steps 20 --warmup 5 --no-cpu --spot 0 --trajectory 20"
S="--instance ssn --scenarios 100000 --vertices 16384 --steps 8 --warmup 1 --no-cpu --spot 0 --trajectory 8"
bash tools/gpu_session.sh gpurun_out/s9 \
  "tests|300|python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "storm_lf|150|python bench.py $A > gpurun_out/s9/storm_lf.json" \
  "storm_plain|150|TWOSD_LONG_FIRST=0 python bench.py $A > gpurun_out/s9/storm_plain.json" \
  "ssn_lf|200|python bench.py $S > gpurun_out/s9/ssn_lf.json" \
  "ssn_plain|200|TWOSD_LONG_FIRST=0 python bench.py $S > gpurun_out/s9/ssn_plain.json"

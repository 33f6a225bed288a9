#!/bin/bash
# Round-4 session: column-wise pricing for dense rho (ssn) -- GPU tests, then ssn and storm with
# it and without it (TWOSD_PRICE_CW=-1)
S="--instance ssn --scenarios 100000 --vertices 16384 --steps 8 --warmup 1 --no-cpu --spot 0 --trajectory 0"
A="--steps 20 --warmup 5 --no-cpu --spot 0 --trajectory 0"
bash tools/gpu_session.sh gpurun_out/s13 \
  "tests|300|python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "ssn_cw|200|python bench.py $S > gpurun_out/s13/ssn_cw.json" \
  "ssn_scatter|200|TWOSD_PRICE_CW=-1 python bench.py $S > gpurun_out/s13/ssn_scatter.json" \
  "storm|150|python bench.py $A > gpurun_out/s13/storm.json"

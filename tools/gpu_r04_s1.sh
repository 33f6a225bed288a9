#!/bin/bash
# Round-4 development session on the GPU box (each step under its own limit; stops at a fault)
bash tools/gpu_session.sh gpurun_out/s2 \
  "tests|420|python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests" \
  "bench|240|python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/s2/bench.json" \
  "phases|200|TWOSD_LIB=stamps python -u tools/lp_phases_bench.py 250000" \
  "ab_default|150|python -u tools/lp_speed.py storm 200000 3 && python -u tools/main_pivots.py 250000" \
  "ab_qpf|150|TWOSD_LIB=qpf python -u tools/lp_speed.py storm 200000 3 && TWOSD_LIB=qpf python -u tools/main_pivots.py 250000" \
  "passes2|200|python bench.py --gpus 1 --steps 8 --warmup 4 --no-cpu --spot 0 --trajectory 0 --refresh-passes 2 > gpurun_out/s2/passes2.json"

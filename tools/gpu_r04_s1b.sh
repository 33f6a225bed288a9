#!/bin/bash
# Round-4 session 1b: the register-pressure fix (main) vs without the pipelined queue claim (noq)
bash tools/gpu_session.sh gpurun_out/s5 \
  "tests|420|python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests" \
  "bench|240|python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/s5/bench.json" \
  "ab_main|150|python -u tools/lp_speed.py storm 200000 3 && python -u tools/main_pivots.py 250000" \
  "ab_noq|150|TWOSD_LIB=noq python -u tools/lp_speed.py storm 200000 3 && TWOSD_LIB=noq python -u tools/main_pivots.py 250000"

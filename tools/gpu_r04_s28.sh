#!/bin/bash
# Round-4: the ssn cut at full rounds with 3 blocks per CU against the C oracle
bash tools/gpu_session.sh gpurun_out/s28 \
  "test|300|python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/test_gpu_cut.py -k ssn_full_rounds"

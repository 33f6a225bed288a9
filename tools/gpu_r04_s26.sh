#!/bin/bash
# Round-4 A/B: the cut kernel at 3 blocks per CU for KB <= 22 (ssn) -- parity tests on the variant, then ssn configs
C="--instance ssn --scenarios 100000 --no-cpu --steps 8 --warmup 1 --trajectory 0 --spot 1024"
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu"
bash tools/gpu_session.sh gpurun_out/s26 \
  "tests_lb3|300|TWOSD_LIB=lb3 $T tests/test_gpu_cut.py" \
  "base16k|200|python bench.py $C --vertices 16384 > gpurun_out/s26/base16k.json" \
  "lb3_16k|200|TWOSD_LIB=lb3 python bench.py $C --vertices 16384 > gpurun_out/s26/lb3_16k.json" \
  "base64k|200|python bench.py $C --vertices 65536 > gpurun_out/s26/base64k.json" \
  "lb3_64k|200|TWOSD_LIB=lb3 python bench.py $C --vertices 65536 > gpurun_out/s26/lb3_64k.json"

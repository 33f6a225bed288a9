#!/bin/bash
# Round-6 GPU pass O: the fp32 argmax with the previous chunk's test interleaved with the MFMAs
# (TWOSD_CUT3_IL=1, build il1): cut parity tests on it, then the cut alone (storm 1M at x_EV,
# |V| = 4096) under a kernel trace, default against il1.
set -u
mkdir -p gpurun_out/r06o
export TMPDIR=/tmp
TWOSD_LIB=il1 timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_cut.py tests/test_gpu_configs.py > gpurun_out/r06o/tests.log 2>&1 || { tail -30 gpurun_out/r06o/tests.log; exit 1; }
tail -1 gpurun_out/r06o/tests.log
for L in default il1; do
  LV=$L; [ $L = default ] && LV=
  TWOSD_LIB=$LV timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r06o/$L -o run --output-format csv -- python3 tools/cut_speed.py 1000000 4096 5 > gpurun_out/r06o/$L.json 2> gpurun_out/r06o/$L.err || { tail -5 gpurun_out/r06o/$L.err; exit 1; }
  tail -1 gpurun_out/r06o/$L.json | cut -c1-200
done

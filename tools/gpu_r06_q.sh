#!/bin/bash
# Round-6 GPU pass Q: the fp32 argmax's candidate steps (prefilter masks, one passing vertex per row
# and lane per round): cut parity tests on the default build and the HOLD build (first log entry in a
# register at 3 blocks per CU), the prefilter counters (cnt build), then the cut alone under a kernel
# trace and the storm driver protocol (default, hold) and ssn |V| = 16384.
set -u
mkdir -p gpurun_out/r06q
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_cut.py tests/test_gpu_configs.py > gpurun_out/r06q/tests.log 2>&1 || { tail -30 gpurun_out/r06q/tests.log; exit 1; }
tail -1 gpurun_out/r06q/tests.log
TWOSD_LIB=hold timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_cut.py > gpurun_out/r06q/tests_hold.log 2>&1 || { tail -30 gpurun_out/r06q/tests_hold.log; exit 1; }
tail -1 gpurun_out/r06q/tests_hold.log
TWOSD_LIB=cnt TWOSD_CUT3_COUNT_PRINT=1 timeout -k 10 200 python3 tools/cut_speed.py 1000000 4096 2 2>&1 | tail -2 | cut -c1-200
for L in default hold; do
  LV=$L; [ $L = default ] && LV=
  TWOSD_LIB=$LV timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r06q/$L -o run --output-format csv -- python3 tools/cut_speed.py 1000000 4096 5 > gpurun_out/r06q/$L.json 2> gpurun_out/r06q/$L.err || { tail -5 gpurun_out/r06q/$L.err; exit 1; }
  tail -1 gpurun_out/r06q/$L.json | cut -c1-200
done
bash tools/ab_bench.sh r06q/ab "" "TWOSD_LIB=hold" "--instance ssn --scenarios 100000 --vertices 16384" || exit 1

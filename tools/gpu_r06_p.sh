#!/bin/bash
# Round-6 GPU pass P: the fp32 argmax with an fp32 prefilter (bases rounded up, floors rounded down)
# in place of the fp64 per-score test, fp64 bases of the rare path staged in an LDS ring: cut parity
# tests, then the cut alone (storm 1M at x_EV, |V| = 4096) under a kernel trace (default build and
# noslp: no packed fp32 adds), then the storm driver protocol and ssn |V| = 16384.
set -u
mkdir -p gpurun_out/r06p
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_cut.py tests/test_gpu_configs.py > gpurun_out/r06p/tests.log 2>&1 || { tail -30 gpurun_out/r06p/tests.log; exit 1; }
tail -1 gpurun_out/r06p/tests.log
for L in default noslp; do
  LV=$L; [ $L = default ] && LV=
  TWOSD_LIB=$LV timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r06p/$L -o run --output-format csv -- python3 tools/cut_speed.py 1000000 4096 5 > gpurun_out/r06p/$L.json 2> gpurun_out/r06p/$L.err || { tail -5 gpurun_out/r06p/$L.err; exit 1; }
  tail -1 gpurun_out/r06p/$L.json | cut -c1-200
done
bash tools/ab_bench.sh r06p/ab "" "TWOSD_LIB=noslp" "--instance ssn --scenarios 100000 --vertices 16384" || exit 1

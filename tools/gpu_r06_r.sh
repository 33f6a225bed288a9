#!/bin/bash
# Round-6 GPU pass R: what the fp32 argmax's per-chunk barrier costs now (diagnostic build dnosync:
# chunk c_lo reused, no barrier; results invalid, timing only) and the 2-blocks-per-CU build (b2),
# against the default build: the cut alone (storm 1M at x_EV, |V| = 4096) under a kernel trace.
set -u
mkdir -p gpurun_out/r06r
export TMPDIR=/tmp
for L in dnosync; do
  LV=$L; [ $L = default ] && LV=
  TWOSD_LIB=$LV timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r06r/$L -o run --output-format csv -- python3 tools/cut_speed.py 1000000 4096 5 > gpurun_out/r06r/$L.json 2> gpurun_out/r06r/$L.err || { tail -5 gpurun_out/r06r/$L.err; exit 1; }
  tail -1 gpurun_out/r06r/$L.json | cut -c1-150
done

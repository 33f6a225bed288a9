#!/bin/bash
# Round-6 GPU pass N: where the fp32 argmax's time goes -- the cut alone (storm 1M at x_EV, |V| = 4096)
# under a kernel trace, on diagnostic builds (results invalid, timing only): no per-chunk barrier /
# staging, no score epilogue, neither; against the default build.
set -u
mkdir -p gpurun_out/r06n
export TMPDIR=/tmp
for L in default dnosync dnofin dboth; do
  LV=$L; [ $L = default ] && LV=
  TWOSD_LIB=$LV timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r06n/$L -o run --output-format csv -- python3 tools/cut_speed.py 1000000 4096 5 > gpurun_out/r06n/$L.json 2> gpurun_out/r06n/$L.err || { tail -5 gpurun_out/r06n/$L.err; exit 1; }
  tail -1 gpurun_out/r06n/$L.json | cut -c1-200
  find gpurun_out/r06n/$L -name '*kernel_stats.csv' -exec grep -h "argmax3\|fixup\|tail_merge" {} \; | cut -d, -f1-4
done

#!/bin/bash
# Round-6 GPU pass S: fp32 argmax fragment-group size (KG = 3 / 6 (default) / 10 / 15 k-blocks read
# ahead) and no scheduling barrier between groups (sb0), on the current argmax: the cut alone
# (storm 1M at x_EV, |V| = 4096) under a kernel trace.
set -u
mkdir -p gpurun_out/r06s
export TMPDIR=/tmp
for L in default kg3 kg10 kg15 sb0; do
  LV=$L; [ $L = default ] && LV=
  TWOSD_LIB=$LV timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r06s/$L -o run --output-format csv -- python3 tools/cut_speed.py 1000000 4096 4 > gpurun_out/r06s/$L.json 2> gpurun_out/r06s/$L.err || { tail -5 gpurun_out/r06s/$L.err; exit 1; }
  tail -1 gpurun_out/r06s/$L.json | cut -c1-120
done

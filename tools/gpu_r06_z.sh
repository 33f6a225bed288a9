#!/bin/bash
# Round-6 GPU pass Z: the cut fixup's grid (TWOSD_FIX_BPC = blocks per CU: 2 / 3 / 4 (default) / 8),
# the cut alone (storm 1M at x_EV, |V| = 4096) under a kernel trace.
set -u
mkdir -p gpurun_out/r06z
export TMPDIR=/tmp
for B in 2 3 4 8; do
  TWOSD_FIX_BPC=$B timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r06z/b$B -o run --output-format csv -- python3 tools/cut_speed.py 1000000 4096 4 > gpurun_out/r06z/b$B.json 2> gpurun_out/r06z/b$B.err || { tail -5 gpurun_out/r06z/b$B.err; exit 1; }
  tail -1 gpurun_out/r06z/b$B.json | cut -c1-100
done

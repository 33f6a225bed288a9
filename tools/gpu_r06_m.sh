#!/bin/bash
# Round-6 GPU pass M: refresh pool size on the storm driver protocol, now that the pool build copies
# untouched columns (4096 default; 5120 / 6144 bases; 6144 from 16384 training scenarios).
set -u
bash tools/ab_bench.sh r06m "" "--refresh-pool 5120" "--refresh-pool 6144" "--refresh-pool 6144 --refresh-train 16384" || exit 1
cat gpurun_out/r06m.txt

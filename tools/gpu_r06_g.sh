#!/bin/bash
# Round-6 GPU pass G: fp32 cut pass A/B -- fragment groups (KG = 6 / 10 / 15 k-blocks read ahead)
# and the scheduling barrier between them, on the storm driver protocol.
set -u
bash tools/ab_bench.sh r06g "" "TWOSD_LIB=kg10" "TWOSD_LIB=kg15" "TWOSD_LIB=sb0" || exit 1
cat gpurun_out/r06g.txt

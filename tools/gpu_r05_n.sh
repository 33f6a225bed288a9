#!/bin/bash
# Round-5 GPU pass N: A/B of the candidate lists' training count, then the final profile session
# of the driver's command (kernel trace + PMC passes, tools/profile_r04.sh r05final).
set -u
mkdir -p gpurun_out
bash tools/ab_bench.sh r05_candtrain "" "--refresh-cand-train 8192" "--refresh-cand-train 4096" || exit 1
cat gpurun_out/r05_candtrain.txt
bash tools/profile_r04.sh r05final

#!/bin/bash
# Round-6 GPU pass B: eta-group size A/B (EG = 1 / 2 / 4 etas per memory round trip in BTRAN / FTRAN)
# and the refresh pool size on ssn 100k (|V| = 16384), then EG on the storm driver protocol.
set -u
S="--instance ssn --scenarios 100000 --vertices 16384"
bash tools/ab_bench.sh r06b_ssn "$S" "TWOSD_LIB=eg1 $S" "TWOSD_LIB=eg4 $S" "$S --refresh-pool 1024" "$S --refresh-pool 2048" || exit 1
cat gpurun_out/r06b_ssn.txt
bash tools/ab_bench.sh r06b_storm "" "TWOSD_LIB=eg1" "TWOSD_LIB=eg4" || exit 1
cat gpurun_out/r06b_storm.txt

#!/bin/bash
# Round-6 GPU pass C: ssn 100k (|V| = 16384) warm-start pool / selection A/B on the driver protocol.
set -u
S="--instance ssn --scenarios 100000 --vertices 16384"
bash tools/ab_bench.sh r06c_ssn "$S --refresh-pool 2048 --pool-level1 0" "$S --refresh-pool 1024 --pool-level1 0" \
  "$S --refresh-pool 2048 --refresh-train 4096" "$S --refresh-pool 4096 --refresh-train 8192" \
  "$S --refresh-pool 2048 --pool-level1 256 --pool-cands 256" "$S --refresh-pool 4096 --refresh-train 16384" || exit 1
cat gpurun_out/r06c_ssn.txt

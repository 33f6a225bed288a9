#!/bin/bash
# Round-6 GPU pass V: ssn |V| = 16384 refresh sizes on the push-full-mode build (pool 1024 / 2048
# (default) / 4096 bases; 2048 bases from 4096 training scenarios instead of 8192), driver protocol.
set -u
S="--instance ssn --scenarios 100000 --vertices 16384"
bash tools/ab_bench.sh r06v/ab "$S" "$S --refresh-pool 1024" "$S --refresh-pool 4096" "$S --refresh-train 4096" || exit 1

#!/bin/bash
# Round-5 GPU pass O: N = 8 per-rank emulation with more refresh training scenarios (the candidate
# lists come from them): pool 2048 with 16384 training scenarios, pool 3072 with 16384.
set -u
mkdir -p gpurun_out
for cfg in "2048 16384" "3072 16384"; do
  set -- $cfg
  timeout -k 10 600 python3 -u tools/shard_emulate.py 8 1000000 20 $1 $2 5 > gpurun_out/r05o_n8_$1_$2.txt 2> gpurun_out/r05o_n8_$1_$2.err || { tail -5 gpurun_out/r05o_n8_$1_$2.err; exit 1; }
  tail -1 gpurun_out/r05o_n8_$1_$2.txt
done

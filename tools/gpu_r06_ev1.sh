#!/bin/bash
# Round-6 evidence pass 1 (final build): the other BASELINE configs (tools/configs_r06.sh), the N = 8
# per-rank step emulated on one GPU (tools/shard_emulate.py), and the N = 2 rehearsal of the bench's
# multi-rank path (tools/rehearse_n2.sh).
set -u
mkdir -p gpurun_out
bash tools/configs_r06.sh || exit 1
timeout -k 10 600 python3 -u tools/shard_emulate.py 8 1000000 20 2048 8192 5 > gpurun_out/r06_n8.txt 2> gpurun_out/r06_n8.err || { tail -5 gpurun_out/r06_n8.err; exit 1; }
tail -1 gpurun_out/r06_n8.txt
bash tools/rehearse_n2.sh > gpurun_out/r06_rehearse_n2.txt 2>&1 || { tail -20 gpurun_out/r06_rehearse_n2.txt; exit 1; }
cat gpurun_out/r06_rehearse_n2.txt

#!/bin/bash
# Round-6 GPU pass Y: LP queue order with the rarest pool bases first (TWOSD_ORDER_DESC=1; the last
# scenarios of the queue are then the common, short ones) against the default order: storm driver
# protocol, then the N = 8 per-rank step emulated on one GPU, both orders.
set -u
mkdir -p gpurun_out/r06y
bash tools/ab_bench.sh r06y/ab "" "TWOSD_ORDER_DESC=1" || exit 1
timeout -k 10 600 python3 -u tools/shard_emulate.py 8 1000000 20 2048 8192 5 > gpurun_out/r06y/n8_default.txt 2> gpurun_out/r06y/n8_default.err || { tail -5 gpurun_out/r06y/n8_default.err; exit 1; }
tail -1 gpurun_out/r06y/n8_default.txt
TWOSD_ORDER_DESC=1 timeout -k 10 600 python3 -u tools/shard_emulate.py 8 1000000 20 2048 8192 5 > gpurun_out/r06y/n8_desc.txt 2> gpurun_out/r06y/n8_desc.err || { tail -5 gpurun_out/r06y/n8_desc.err; exit 1; }
tail -1 gpurun_out/r06y/n8_desc.txt

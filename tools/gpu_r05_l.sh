#!/bin/bash
# Round-5 GPU pass L: the N = 8 per-rank emulation again (after the PK / twin maintenance change),
# then a kernel trace of a shorter emulation (per-kernel times of the 125k-scenario shards).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
echo "n8 emulation"
timeout -k 10 600 python3 -u tools/shard_emulate.py 8 1000000 20 2048 8192 5 > gpurun_out/r05l_n8.txt 2> gpurun_out/r05l_n8.err || { tail -5 gpurun_out/r05l_n8.err; exit 1; }
tail -2 gpurun_out/r05l_n8.txt
echo "n8 trace"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/r05l_tr -o run --output-format csv -- python3 tools/shard_emulate.py 8 1000000 4 2048 8192 4 > gpurun_out/r05l_tr.txt 2> gpurun_out/r05l_tr.err || { tail -5 gpurun_out/r05l_tr.err; exit 1; }
python3 tools/prof_reduce.py gpurun_out/r05l_tr gpurun_out/r05l_tr > /dev/null

#!/bin/bash
# One GPU session: full bench (+CPU baseline), rocprofv3 kernel-trace stats, and separate
# PMC passes for HBM traffic (FETCH_SIZE / WRITE_SIZE), all under their own time limits.
# Usage (from the repo root, on the GPU box): bash tools/profile_round.sh <tag> [scenarios]
set -u
TAG=${1:-r01}
NS=${2:-1000000}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 420 python bench.py --scenarios $NS > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed $?"; exit 1; }
tail -1 $OUT/bench.json
timeout -k 10 420 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py --scenarios $NS --steps 2 --warmup 1 --no-cpu > $OUT/trace_bench.json 2> $OUT/trace.err || { echo "trace failed $?"; exit 1; }
timeout -k 10 420 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch -o run --output-format csv -- python3 bench.py --scenarios $NS --steps 1 --warmup 0 --no-cpu > /dev/null 2> $OUT/pmc_fetch.err || { echo "pmc fetch failed $?"; exit 1; }
timeout -k 10 420 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write -o run --output-format csv -- python3 bench.py --scenarios $NS --steps 1 --warmup 0 --no-cpu > /dev/null 2> $OUT/pmc_write.err || { echo "pmc write failed $?"; exit 1; }
echo done

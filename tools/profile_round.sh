#!/bin/bash
# One GPU session: full bench (+CPU baseline, spot check), rocprofv3 kernel-trace stats of a
# short run, and separate PMC passes (HBM traffic: FETCH_SIZE, WRITE_SIZE; fp64 MFMA: ops,
# busy cycles), every step under its own time limit.
# Usage (from the repo root, on the GPU box): bash tools/profile_round.sh <tag> [scenarios]
set -u
TAG=${1:-r02}
NS=${2:-1000000}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
SHORT="--scenarios $NS --no-cpu --spot 0"
timeout -k 10 600 python bench.py --scenarios $NS > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed $?"; exit 1; }
tail -1 $OUT/bench.json | cut -c1-400
timeout -k 10 420 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py $SHORT --steps 4 --warmup 1 > $OUT/trace_bench.json 2> $OUT/trace.err || { echo "trace failed $?"; exit 1; }
timeout -k 10 420 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch -o run --output-format csv -- python3 bench.py $SHORT --steps 1 --warmup 0 > /dev/null 2> $OUT/pmc_fetch.err || { echo "pmc fetch failed $?"; exit 1; }
timeout -k 10 420 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write -o run --output-format csv -- python3 bench.py $SHORT --steps 1 --warmup 0 > /dev/null 2> $OUT/pmc_write.err || { echo "pmc write failed $?"; exit 1; }
timeout -k 10 420 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_INSTS_VALU_MFMA_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $OUT/pmc_mfma -o run --output-format csv -- python3 bench.py $SHORT --steps 1 --warmup 0 > /dev/null 2> $OUT/pmc_mfma.err || { echo "pmc mfma failed $?"; exit 1; }
echo done

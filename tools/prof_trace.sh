#!/bin/bash
# One rocprofv3 kernel-trace/stats pass of bench.py on the GPU box (quick per-kernel timing),
# reduced on the box by tools/prof_reduce.py.  Usage (repo root): bash tools/prof_trace.sh <tag> [bench args]
# Default bench args: the driver's protocol without the CPU baseline / spot check / trajectory.
set -u
TAG=${1:-trace}; shift || true
ARGS=${*:-"--gpus 1 --steps 20 --warmup 5 --no-cpu --spot 0 --trajectory 0"}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 420 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py $ARGS > $OUT/bench.json 2> $OUT/trace.err
rc=$?
echo "trace rc=$rc $(tail -c 300 $OUT/bench.json | tr -d '\n' | cut -c1-200)"
[ $rc -eq 0 ] || { tail -5 $OUT/trace.err; exit $rc; }
python3 tools/prof_reduce.py $OUT/trace $OUT/trace

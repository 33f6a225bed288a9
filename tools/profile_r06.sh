#!/bin/bash
# Round-6 profile session on the GPU box: the driver's command (bench.py --gpus 1 --steps 20
# --warmup 5) under rocprofv3 -- a kernel-trace/stats run and separate PMC passes (HBM bytes:
# FETCH_SIZE, WRITE_SIZE; fp64 MFMA; two SQ instruction / wait passes) -- each step under its own
# time limit, reduced on the box by tools/prof_reduce.py; tools/pmc_timed.py then keeps the timed steps' launches per x point.
# Usage (repo root, GPU box): bash tools/profile_r06.sh <tag> [bench args, e.g. --instance ssn --scenarios 100000 --vertices 16384]
set -u
TAG=${1:-r06}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
ARGS="--gpus 1 --steps 20 --warmup 5 --no-cpu --spot 0 --trajectory 0 $*"
run() {   # run <name> <seconds> <rocprofv3 args...>
    local name=$1 secs=$2; shift 2
    timeout -k 10 $secs rocprofv3 "$@" -d $OUT/$name -o run --output-format csv -- python3 bench.py $ARGS > $OUT/${name}_bench.json 2> $OUT/$name.err
    local rc=$?
    echo "$name rc=$rc $(tail -c 300 $OUT/${name}_bench.json | tr -d '\n' | cut -c1-200)"
    tail -3 $OUT/$name.err
    [ $rc -eq 0 ] || exit $rc
    python3 tools/prof_reduce.py $OUT/$name $OUT/$name   # raw per-dispatch CSVs exceed the copy-back limit
}
run trace 420 --kernel-trace --stats
run pmc_fetch 420 --pmc FETCH_SIZE
run pmc_write 420 --pmc WRITE_SIZE
run pmc_mfma 420 --pmc SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_INSTS_VALU_MFMA_F32 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE
run pmc_sq1 420 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU
run pmc_sq2 420 --pmc SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_MISC
echo done

#!/bin/bash
# Round-end check on the GPU box: the gpu test suite, smoke(), the rocprof profile set
# (tools/profile_round.sh) and its PMC summary.  Each GPU step runs under its own time limit;
# the script stops at the first failing step (a fault, abort or time limit ends the GPU work).
# Usage: bash tools/gpu_round_check.sh <round tag, e.g. r03>
set -u
TAG=${1:?round tag}
mkdir -p gpurun_out
step() {   # step <name> <log> <cmd...>
    local name=$1 log=$2; shift 2
    "$@" > "$log" 2>&1
    local rc=$?
    echo "$name rc=$rc"; tail -3 "$log"
    if [ $rc -ne 0 ]; then echo "stopping after $name"; exit $rc; fi
}
step tests gpurun_out/gt.log timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests
step smoke gpurun_out/smoke.log timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()"
step profile gpurun_out/prof.log bash tools/profile_round.sh "$TAG"
step summary gpurun_out/sum.log python3 tools/pmc_summarize.py "gpurun_out/$TAG" "gpurun_out/${TAG}_summary" 1000000

#!/bin/bash
# Round-6 GPU pass W: two-level candidate lists from the training scenarios' own optimal bases
# (TWOSD_CAND_OPT=1: no flat selection over the pool) against the flat picks (default), storm driver
# protocol and ssn |V| = 16384; refresh parity tests first.
set -u
mkdir -p gpurun_out/r06w
TWOSD_CAND_OPT=1 timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_pool_refresh.py > gpurun_out/r06w/tests.log 2>&1 || { tail -30 gpurun_out/r06w/tests.log; exit 1; }
tail -1 gpurun_out/r06w/tests.log
S="--instance ssn --scenarios 100000 --vertices 16384"
bash tools/ab_bench.sh r06w/ab "" "TWOSD_CAND_OPT=1" "$S" "TWOSD_CAND_OPT=1 $S" || exit 1

#!/bin/bash
# Round-6 GPU pass T: the selection streams' last records as one partial batch (seltb; seltb32: 32-record
# batches) against the default build: selection parity tests, then the storm driver protocol.
set -u
mkdir -p gpurun_out/r06t
TWOSD_LIB=seltb timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_pool_refresh.py tests/test_gpu_lp.py tests/test_gpu_dist.py > gpurun_out/r06t/tests.log 2>&1 || { tail -30 gpurun_out/r06t/tests.log; exit 1; }
tail -1 gpurun_out/r06t/tests.log
bash tools/ab_bench.sh r06t/ab "" "TWOSD_LIB=seltb" "TWOSD_LIB=seltb32" "" || exit 1

#!/bin/bash
# Round-6 GPU pass X: the ratio test's first pass over the slots the pricing wrote only
# (TWOSD_HARRIS_MASK=1, build hmask): LP parity / determinism tests on it, then the storm driver
# protocol and ssn |V| = 16384 against the default build.
set -u
mkdir -p gpurun_out/r06x
TWOSD_LIB=hmask timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_lp.py tests/test_gpu_vkey.py tests/test_gpu_parity_paths.py tests/test_gpu_configs.py > gpurun_out/r06x/tests.log 2>&1 || { tail -30 gpurun_out/r06x/tests.log; exit 1; }
tail -1 gpurun_out/r06x/tests.log
S="--instance ssn --scenarios 100000 --vertices 16384"
bash tools/ab_bench.sh r06x/ab "" "TWOSD_LIB=hmask" "$S" "TWOSD_LIB=hmask $S" || exit 1

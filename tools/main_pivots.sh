#!/bin/bash
# main-solve pivot distribution per bench x point (tools/main_pivots.py), 250k scenarios
mkdir -p gpurun_out
timeout -k 10 300 python tools/main_pivots.py 250000 4096 > gpurun_out/mp.log 2>&1 || exit 1
tail -4 gpurun_out/mp.log

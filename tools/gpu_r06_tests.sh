#!/bin/bash
# Round-6 GPU check: the whole GPU suite (durations of the slowest tests), then smoke().
set -u
mkdir -p gpurun_out
T=${1:-r06}
timeout -k 10 900 python3 -u -m pytest --maxfail=10 -q --durations=15 --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/${T}_tests.log 2>&1 || { tail -60 gpurun_out/${T}_tests.log; exit 1; }
tail -25 gpurun_out/${T}_tests.log
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || { tail -5 gpurun_out/${T}_smoke.log; exit 1; }
tail -1 gpurun_out/${T}_smoke.log

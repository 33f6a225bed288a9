#!/bin/bash
# Round-5 GPU pass F: storm warm-start hindsight at x_EV and SD-4 with the per-(basis, scenario)
# pivot tables dumped for an offline study of the selection key (tools/ssn_hindsight.py).
set -u
mkdir -p gpurun_out
HINDSIGHT_DUMP=gpurun_out/hs timeout -k 10 900 python3 -u tools/ssn_hindsight.py 96 16 0,4 storm > gpurun_out/r05f_storm_hindsight.txt 2> gpurun_out/r05f_storm.err || { tail -3 gpurun_out/r05f_storm.err; exit 1; }
cat gpurun_out/r05f_storm_hindsight.txt

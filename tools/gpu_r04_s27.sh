#!/bin/bash
# Round-4: N = 2 rehearsal of the bench's multi-rank path on the closing tree (both ranks on cuda:0, gloo)
mkdir -p gpurun_out/s27
timeout -k 10 800 bash tools/rehearse_n2.sh 200000 > gpurun_out/s27/rehearse_n2.txt 2>&1
rc=$?; cat gpurun_out/s27/rehearse_n2.txt; exit $rc

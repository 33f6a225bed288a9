#!/bin/bash
# Development A/B of LP kernel builds on the GPU box: bash tools/ab_lp.sh "<variants>" (""=default)
# per variant: fixed-work LP timing (lp_speed, primary basis), pivot-path agreement with the C
# oracle (pivot_parity) and the bench protocol's LP time per x point (main_pivots, 250k).
set -o pipefail
mkdir -p gpurun_out
for v in $1; do
  [ "$v" = "default" ] && v=""
  TWOSD_LIB=$v timeout -k 10 150 python -u tools/lp_speed.py storm 200000 3 > gpurun_out/ls_$v.txt 2>&1 || { tail -5 gpurun_out/ls_$v.txt; exit 1; }
  grep "N=" gpurun_out/ls_$v.txt | cut -c1-110
  TWOSD_LIB=$v timeout -k 10 100 python -u tools/pivot_parity.py 3000 > gpurun_out/pp_$v.txt 2>&1 || { tail -5 gpurun_out/pp_$v.txt; exit 1; }
  grep "N=" gpurun_out/pp_$v.txt
  TWOSD_LIB=$v timeout -k 10 200 python -u tools/main_pivots.py 250000 > gpurun_out/mp_$v.txt 2>&1 || { tail -5 gpurun_out/mp_$v.txt; exit 1; }
  grep -o "x[0-9]*: mean [0-9.]*\|LP [0-9.]* ms" gpurun_out/mp_$v.txt | paste -s -d' '
done

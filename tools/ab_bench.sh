#!/bin/bash
# A/B of bench.py options on the GPU box: each variant runs the driver's protocol (steps 20, warmup 5,
# no CPU baseline / spot check / trajectory unless the variant asks) and one summary line per variant
# goes to gpurun_out/<tag>.txt (full JSON lines to <tag>.jsonl).
# Usage (repo root): bash tools/ab_bench.sh <tag> "<variant args>" ["<variant args>" ...]   ("" = defaults;
# NAME=value tokens of a variant go to its environment, e.g. "TWOSD_LIB=xu2 --refresh-passes 2")
set -u
TAG=$1; shift
mkdir -p gpurun_out
OUT=gpurun_out/$TAG
: > $OUT.txt; : > $OUT.jsonl
for v in "$@"; do
  envs=(); args=()
  for tok in $v; do   # NAME=value tokens (not options) set the environment of the variant (e.g. TWOSD_LIB=xu2)
    if [[ $tok == *=* && $tok != -* ]]; then envs+=("$tok"); else args+=("$tok"); fi
  done
  timeout -k 10 300 env "${envs[@]}" python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --spot 0 --trajectory 0 "${args[@]}" > $OUT.cur 2> $OUT.err
  rc=$?
  if [ $rc -ne 0 ]; then echo "variant [$v] rc=$rc" >> $OUT.txt; tail -5 $OUT.err >> $OUT.txt; exit $rc; fi
  tail -1 $OUT.cur >> $OUT.jsonl
  python3 - "$v" $OUT.cur >> $OUT.txt <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
ph = d["phases_ms_per_step"]
xs = " ".join(f"[{p['x'][:6]} {p['ms_per_step']:.1f}ms ref {p['pool_refresh_ms']:.1f} lp {p['lp_kernel_ms']:.1f} piv {p['lp_pivots_mean']:.2f}]" for p in d["x_points"])
print(f"[{sys.argv[1]}] {d['ms_per_step']:.2f} ms/step {d['value']/1e6:.2f} M/s | lp {ph['lp_kernel']:.1f} sel {ph['pool_select']:.1f} "
      f"cut {ph['cut_partial']:.1f} | piv {d['lp_pivots_mean']:.2f} | {xs}")
PY
  tail -1 $OUT.txt
done

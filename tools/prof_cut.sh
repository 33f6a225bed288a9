#!/bin/bash
# Kernel trace of tools/cut_speed.py (storm 1M at x_EV, |V| = 4096): per-kernel durations of the cut.
# Usage (GPU box, repo root): bash tools/prof_cut.sh <tag> [N] [|V|] [reps]
set -u
TAG=${1:-cut}; shift || true
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 tools/cut_speed.py ${1:-1000000} ${2:-4096} ${3:-3} > $OUT/cut.json 2> $OUT/trace.err
rc=$?
tail -1 $OUT/cut.json
[ $rc -eq 0 ] || { tail -5 $OUT/trace.err; exit $rc; }
python3 tools/prof_reduce.py $OUT/trace $OUT/trace
python3 - $OUT/trace_trace.csv.gz <<'PY'
import csv, gzip, sys, collections
rows = list(csv.DictReader(gzip.open(sys.argv[1], "rt")))
d = collections.defaultdict(list)
for r in rows:
    if "cut_" in r["Kernel_Name"]:
        d[r["Kernel_Name"].split("(")[0].split("::")[-1]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
for k, v in d.items():
    print(k, len(v), [round(x, 3) for x in v[-3:]])
PY

#!/bin/bash
# Round-5 GPU pass I: cut parity tests, the cut alone at 1M, and its WRITE_SIZE / FETCH_SIZE per
# launch (one PMC pass each over tools/cut_speed.py).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
echo "cut tests"
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_cut.py tests/test_gpu_large_v.py tests/test_gpu_julia_mirror.py > gpurun_out/r05i_tests.log 2>&1 || { tail -30 gpurun_out/r05i_tests.log; exit 1; }
tail -2 gpurun_out/r05i_tests.log
echo "cut speed"
timeout -k 10 200 python3 -u tools/cut_speed.py 1000000 4096 5 || exit 1
for c in WRITE_SIZE FETCH_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c -d gpurun_out/r05i_$c -o run --output-format csv -- python3 tools/cut_speed.py 1000000 4096 3 > gpurun_out/r05i_$c.log 2>&1 || { tail -5 gpurun_out/r05i_$c.log; exit 1; }
  python3 - "$c" <<'PY'
import csv, glob, sys
c = sys.argv[1]
f = glob.glob(f"gpurun_out/r05i_{c}/**/*counter_collection.csv", recursive=True)[0]
rows = [r for r in csv.DictReader(open(f)) if "cut_argmax2" in r["Kernel_Name"] or "cut_fixup" in r["Kernel_Name"]]
by = {}
for r in rows:
    by.setdefault((r["Kernel_Name"][:40], r["Dispatch_Id"]), 0.0)
    by[(r["Kernel_Name"][:40], r["Dispatch_Id"])] += float(r["Counter_Value"])
for k, v in list(by.items())[-4:]:
    print(c, k[0], round(v * 1024 / 1e6, 1), "MB")
PY
done

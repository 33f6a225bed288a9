#!/bin/bash
# Round-5 GPU pass J: cut parity tests, the storm cut alone, and a kernel trace of the ssn
# |V| = 65536 config (where the cut's time per launch goes on ssn).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
echo "cut tests"
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_cut.py tests/test_gpu_large_v.py tests/test_gpu_julia_mirror.py > gpurun_out/r05j_tests.log 2>&1 || { tail -30 gpurun_out/r05j_tests.log; exit 1; }
tail -2 gpurun_out/r05j_tests.log
echo "cut speed"
timeout -k 10 200 python3 -u tools/cut_speed.py 1000000 4096 5 || exit 1
echo "ssn trace"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r05j_ssn -o run --output-format csv -- python3 bench.py --instance ssn --scenarios 100000 --vertices 65536 --no-cpu --steps 8 --warmup 1 --trajectory 0 --spot 0 > gpurun_out/r05j_ssn.json 2> gpurun_out/r05j_ssn.err || { tail -5 gpurun_out/r05j_ssn.err; exit 1; }
python3 tools/prof_reduce.py gpurun_out/r05j_ssn gpurun_out/r05j_ssn > /dev/null
python3 - <<'PY'
import csv, gzip, glob, collections
f = glob.glob("gpurun_out/r05j_ssn/*trace*.csv.gz")[0]
d = collections.defaultdict(list)
for r in csv.DictReader(gzip.open(f, "rt")):
    d[r["Kernel_Name"].split("(")[0][-40:]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
for n, v in sorted(d.items(), key=lambda kv: -sum(kv[1][-8:]))[:14]:
    print(f"{n:42s} n={len(v):4d} last8 mean {sum(v[-8:]) / min(8, len(v)):.3f} ms")
PY

#!/bin/bash
# SQ counter passes over one bench step (storm 1M at x_EV, refreshed pool), summed per kernel:
# bash tools/pmc_sq_bench.sh [lib variant or default] [scenarios]
# Each pass is its own rocprofv3 run (at most 8 SQ counters per pass) under its own time limit.
set -u
export TMPDIR=/tmp
LIB=${1:-default}; NS=${2:-1000000}
[ "$LIB" = default ] && LIBV="" || LIBV=$LIB
OUT=gpurun_out/pmc_sq_$LIB
mkdir -p $OUT
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAVES"
P2="SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC"
P3="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_BRANCH SQ_ACTIVE_INST_FLAT SQ_INST_CYCLES_SALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  TWOSD_LIB=$LIBV timeout -s KILL 120 rocprofv3 --pmc $P -d $OUT/p$i -o run --output-format csv -- python3 bench.py --scenarios $NS --no-cpu --spot 0 --steps 1 --warmup 0 > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
python3 - "$OUT" <<'EOP'
import csv, glob, collections, sys
acc = collections.defaultdict(collections.Counter)
for f in sorted(glob.glob(sys.argv[1] + "/p*/**/*counter_collection.csv", recursive=True)):
    for r in csv.DictReader(open(f)):
        k = r.get("Kernel_Name", "").split("(")[0].replace("void ", "").replace("twosd::", "")
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, c in sorted(acc.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0)):
    if c.get("SQ_WAVE_CYCLES", 0) <= 0: continue
    print(k, {n: int(v) for n, v in sorted(c.items())})
EOP

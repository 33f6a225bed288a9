set -e
export TMPDIR=/tmp
OUT=gpurun_out/pmc_lp_cur
mkdir -p $OUT
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAVES"
P2="SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  POOL=512 timeout -s KILL 120 rocprofv3 --pmc $P -d $OUT/p$i -o run --output-format csv -- python3 tools/lp_speed.py storm 200000 1 > $OUT/p$i.log 2>&1
done
python3 - <<'PY'
import csv, glob
for f in sorted(glob.glob('gpurun_out/pmc_lp_cur/p*/**/*counter_collection.csv', recursive=True)):
    agg = {}
    for r in csv.DictReader(open(f)):
        if 'lp_hyper_kernel' not in r['Kernel_Name']: continue
        key = (r['Dispatch_Id'])
        agg.setdefault(key, {})[r['Counter_Name']] = float(r['Counter_Value'])
    big = max(agg.values(), key=lambda d: sum(d.values()))
    print(f, {k: int(v) for k, v in big.items()})
PY

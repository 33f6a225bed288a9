# SQ counter passes over the LP batch alone (storm, pool 512): bash tools/pmc_lp.sh <lib> <N>
set -e
export TMPDIR=/tmp
LIB=${1:-default}; N=${2:-200000}; [ "$LIB" = default ] && LIBV="" || LIBV=$LIB
OUT=gpurun_out/pmc_lp_$LIB
mkdir -p $OUT
timeout -k 10 60 rocprofv3 -L > $OUT/counters.txt 2>&1 || true
grep -o "SQ_[A-Z_0-9]*" $OUT/counters.txt | sort -u > $OUT/sq_names.txt || true
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAVES"
P2="SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  ok=1; for c in $P; do grep -qx $c $OUT/sq_names.txt || { echo "missing $c"; ok=0; }; done
  [ $ok = 1 ] || continue
  TWOSD_LIB=$LIBV POOL=512 timeout -s KILL 120 rocprofv3 --pmc $P -d $OUT/p$i -o run --output-format csv -- python3 tools/lp_speed.py storm $N 1 > $OUT/p$i.log 2>&1
done
echo done

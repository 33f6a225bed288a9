# Development A/B of LP kernel builds: bash tools/ab_run.sh "<variants>" [storm N] [ssn N]
set -e
VARS=${1:-base}
NS=${2:-500000}
NN=${3:-200000}
mkdir -p gpurun_out
for v in $VARS; do
  TWOSD_LIB=$v POOL=512 timeout -k 10 120 python tools/lp_speed.py storm $NS 3 2>&1 | grep -v "^pool" >> gpurun_out/ab.log || true
  [ "$NN" -gt 0 ] && TWOSD_LIB=$v POOL=512 timeout -k 10 120 python tools/lp_speed.py ssn $NN 3 2>&1 | grep -v "^pool" >> gpurun_out/ab.log
done
cat gpurun_out/ab.log

# pool size sweep of the LP batch (selection + LP kernel): bash tools/pool_sweep.sh <lib>
LIB=${1:-cur}
mkdir -p gpurun_out
for cfg in "512 16384" "1024 32768" "2048 65536" "4096 131072"; do
  set -- $cfg
  echo "POOL=$1 TRAIN=$2" >> gpurun_out/pool.log
  TWOSD_LIB=$LIB POOL=$1 POOL_TRAIN=$2 timeout -k 10 200 python tools/lp_speed.py storm 500000 2 >> gpurun_out/pool.log 2>&1 || break
done
cat gpurun_out/pool.log

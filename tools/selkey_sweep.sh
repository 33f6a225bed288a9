# pool selection key sweep: key = sum |infeas| + cw * #infeasible rows
mkdir -p gpurun_out
for cw in 0 1 10 100 1000 100000; do
  echo "cw=$cw" >> gpurun_out/selkey.log
  TWOSD_SEL_CW=$cw TWOSD_LIB=cur POOL=512 timeout -k 10 120 python tools/lp_speed.py storm 500000 2 2>&1 | grep -v "^pool" >> gpurun_out/selkey.log || break
done
cat gpurun_out/selkey.log

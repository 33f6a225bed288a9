mkdir -p gpurun_out
for A in ${SWEEP:-"--pool-cands 160"}; do
  timeout -k 10 300 python bench.py --no-cpu --spot 0 --steps 12 --warmup 4 $A > gpurun_out/sw.json 2> gpurun_out/sw.err || { echo "failed $A"; tail -3 gpurun_out/sw.err; exit 1; }
  python3 -c "
import json;d=json.loads(open('gpurun_out/sw.json').read().strip().splitlines()[-1])
print('$A', round(d['value']/1e6,3), round(d['ms_per_step'],2), {k:round(v,2) for k,v in d['phases_ms_per_step'].items()}, [round(x['lp_pivots_mean'],3) for x in d['x_points']], [round(x['pool_refresh_ms'],1) for x in d['x_points']])"
done

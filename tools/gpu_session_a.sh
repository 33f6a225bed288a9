# development A/B session: bench phases per variant, then (optional) SQ counters of one bench step
# variant token: <lib>[@VAR=value] (lib "default" = libtwosd_hip.so), e.g. "default default@TWOSD_SEL_CW=10"
mkdir -p gpurun_out
for T in $1; do
  L=${T%%@*}; E=""; [ "$T" != "$L" ] && E=$(echo "${T#*@}" | tr "@" " ")
  [ "$L" = default ] && LV="" || LV=$L
  tag=$(echo "$T" | tr -c 'A-Za-z0-9_.\n' '_')
  env TWOSD_LIB=$LV $E timeout -k 10 300 python bench.py --no-cpu --spot 0 --steps 8 --warmup 3 ${BENCH_ARGS:-} > gpurun_out/b_$tag.json 2> gpurun_out/b_$tag.err || { echo "bench $T failed"; tail -5 gpurun_out/b_$tag.err; exit 1; }
  python3 -c "
import json;d=json.loads(open('gpurun_out/b_$tag.json').read().strip().splitlines()[-1])
print('$T', round(d['value']/1e6,3), round(d['ms_per_step'],2), {k:round(v,2) for k,v in d['phases_ms_per_step'].items()}, [round(x['lp_pivots_mean'],4) for x in d['x_points']], [round(x['pool_refresh_ms'],1) for x in d['x_points']])"
done
[ -n "${2:-}" ] && bash tools/pmc_sq_bench.sh $2
exit 0

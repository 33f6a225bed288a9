# bench protocol check: pool refresh log with warmup 4 (TWOSD_DEBUG) and the driver's 20 / 5 run
mkdir -p gpurun_out
TWOSD_DEBUG=1 timeout -k 10 300 python bench.py --no-cpu --spot 0 --steps 4 --warmup 4 > gpurun_out/dbg.json 2> gpurun_out/dbg.err
grep -i "pool_refresh\|pg_assemble\|candidates\|not optimal\|error" gpurun_out/dbg.err | head -60
python3 -c "
import json;d=json.loads(open('gpurun_out/dbg.json').read().strip().splitlines()[-1]); print(d['steps_log']['rows'])"

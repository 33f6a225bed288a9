#!/bin/bash
# The BASELINE.json configs other than the headline, with the round-6 bench protocol (tie rule strict >, no trajectory) (x points
# from an SD run of the instance, per-x pool refresh timed, spot check vs the C oracle; C5 at
# SURVEY's importance scale s = 1.5).  Usage (GPU box, repo root): bash tools/configs_r06.sh
set -u
mkdir -p gpurun_out
OUT=gpurun_out/configs_r06.jsonl
: > $OUT
run() {
  timeout -k 10 400 python bench.py --no-cpu --steps 8 --warmup 1 --trajectory 0 "$@" > gpurun_out/cfg.json 2> gpurun_out/cfg.err || { echo "failed: $*"; tail -5 gpurun_out/cfg.err; return 1; }
  tail -1 gpurun_out/cfg.json >> $OUT
  python3 -c "
import json
d = json.loads(open('gpurun_out/cfg.json').read().strip().splitlines()[-1])
sc = d.get('parity_spot_check') or []
print(d['config']['workload'][:90], '|', round(d['value']), 'subproblems/s', round(d['ms_per_step'], 2), 'ms',
      '| cut', round(d['cutgen']['t_ms'], 2), 'ms', round(d['cutgen']['frac'], 3),
      '| pivots', round(d['lp_pivots_mean'], 2), 'retries', d.get('lp_iter_limit_retries'),
      '| spot max rel err obj', max([x['lp_obj_max_rel_err'] for x in sc] or [None]), 'cut value', max([x['cut_value_rel_err'] for x in sc] or [None]), 'alpha', max([x.get('alpha_rel_err', 0) for x in sc] or [None]), 'beta', max([x.get('beta_max_rel_err', 0) for x in sc] or [None]))"
}
run --instance lands --scenarios 10000 --spot 2048
run --instance ssn --scenarios 100000 --vertices 16384 --spot 2048
run --instance ssn --scenarios 100000 --vertices 65536 --spot 1024
run --instance transship --scenarios 1000000 --epigraphs 4 --importance-scale 1.5 --spot 2048

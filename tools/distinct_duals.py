"""Diagnostic: how many distinct dual vertices (reference push! rule) 1M storm scenarios
produce at the bench configuration, as a function of the number of scenarios pushed."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    from sqlp_amd import smps, twosd
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 1000000
    pool = int(sys.argv[2]) if len(sys.argv) > 2 else 32768
    name = "storm"
    d = os.path.join(ROOT, "data", "smps", name)
    cor, tim, sto = smps.load_smps(d, name)
    sp2 = smps.get_smps_stage_template(cor, tim, 2)
    with open(os.path.join(ROOT, "tests", "golden", "ev_x.json")) as f:
        x = np.array(json.load(f)[name]["x"])
    ctx = twosd.SDContext(sp2, sto)
    ctx.compute_basis(x, smps.mean_values(sto))
    ctx.set_distributions(sto)
    seed = 20250219
    if pool > 1:
        tr = twosd.sdEpigraph(ctx, 1.0, 0.0)
        twosd.add_sampled_scenarios(tr, 4 * pool, seed + 2)
        ctx.pool_build(tr, x, 0, 4 * pool, pool)
        ct = twosd.sdEpigraph(ctx, 1.0, 0.0)
        twosd.add_sampled_scenarios(ct, 262144, seed + 3)
        ctx.pool_build_candidates(ct, x, 0, 262144, 128, 160)
    epi = twosd.sdEpigraph(ctx, 1.0, 0.0)
    twosd.add_sampled_scenarios(epi, N, seed)
    V = twosd.sdDualVertexSet(ctx)
    at, step = 0, 62500
    while at < N:
        twosd.solve_push(epi, x, at, min(step, N - at))
        at += step
        print(f"scenarios {at}: |V| = {len(V)}", flush=True)


if __name__ == "__main__":
    main()

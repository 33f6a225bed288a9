"""Run-to-run determinism of the LP batch and the pool refresh (development check): solve the same
scenarios several times (the work-queue assignment of scenarios to waves differs with timing) and
compare per-scenario status / pivots / objective bits; refresh twice from the same pool and compare.
Usage (GPU box): python tools/lp_repeat.py [N] [reps]"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import bench
    from sqlp_amd import smps, twosd
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 200000
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    name = "storm"
    d = os.path.join(ROOT, "data", "smps", name)
    cor, tim, sto = smps.load_smps(d, name)
    sp2 = smps.get_smps_stage_template(cor, tim, 2)
    with open(os.path.join(ROOT, "tests", "golden", "ev_x.json")) as f:
        x0 = np.array(json.load(f)[name]["x"])
    positions = list(sto.indep.keys())
    import torch
    xs = bench.sd_points(cor, tim, sp2, sto, positions, x0, [0, 4], 20250219 + 7, torch.device("cuda", 0))
    ctx = twosd.SDContext(sp2, sto)
    ctx.compute_basis(x0, smps.mean_values(sto, positions))
    ctx.set_distributions(sto)
    epi = twosd.sdEpigraph(ctx, 1.0, 0.0)
    twosd.add_sampled_scenarios(epi, N, 20250219)
    tr = twosd.sdEpigraph(ctx, 1.0, 0.0)
    twosd.add_sampled_scenarios(tr, 16384, 20250223)
    print("points ready", flush=True)
    for xx in xs:
        print("warm pass", flush=True)
        ctx.pool_refresh(tr, xx, 0, 16384, 4096)
        ctx.pool_build_candidates(tr, xx, 0, 16384, 128, 160)
        twosd.solve_batch(epi, xx, 0, N, want_pi=False)
    xx = xs[0]
    res = []
    for r in range(reps):
        ctx.invalidate_x()
        obj, _, _, st = twosd.solve_batch(epi, xx, 0, N, want_pi=False)
        res.append((obj.view(np.int64).copy(), st.copy(), ctx.last_lp_iters(N)[0].copy(), ctx.last_pool_picks(N).copy()))
    for r in range(1, reps):
        o, s, it, pk = res[r]
        print(json.dumps({"rep": r, "obj_bits_differ": int((o != res[0][0]).sum()), "status_differ": int((s != res[0][1]).sum()),
                          "iters_differ": int((it != res[0][2]).sum()), "picks_differ": int((pk != res[0][3]).sum())}), flush=True)
    # the refresh from one pool, twice (pools saved via the heads; the second from the same start pool)
    heads0 = np.stack([ctx.pool_get(p) for p in range(ctx.pool_size())])
    out = []
    for r in range(2):
        ctx.set_basis(heads0[0])
        for h in heads0[1:]:
            ctx.pool_add_basis(h)
        ctx.pool_refresh(tr, xs[1], 0, 16384, 4096)
        out.append(np.stack([ctx.pool_get(p) for p in range(ctx.pool_size())]))
    same = out[0].shape == out[1].shape and bool((out[0] == out[1]).all())
    print(json.dumps({"refresh_pools_identical": same, "sizes": [o.shape[0] for o in out]}), flush=True)


if __name__ == "__main__":
    main()

"""Pivot distribution of the main solve at every bench x point (storm), after the per-x refresh
the bench does: how much of the LP work sits in the tail, and how many scenarios start at an
optimal pool basis (0 pivots).  Usage (GPU box): python tools/main_pivots.py [scenarios] [pool] [train]"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    torch.cuda.init()
    import bench
    from sqlp_amd import smps, twosd
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 250000
    P = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
    T = int(sys.argv[3]) if len(sys.argv) > 3 else 4 * P
    seed = 20250219
    d = os.path.join(ROOT, "data", "smps", "storm")
    cor, tim, sto = smps.load_smps(d, "storm")
    sp2 = smps.get_smps_stage_template(cor, tim, 2)
    with open(os.path.join(ROOT, "tests", "golden", "ev_x.json")) as f:
        x0 = np.array(json.load(f)["storm"]["x"])
    positions = list(sto.indep.keys())
    xs = bench.sd_points(cor, tim, sp2, sto, positions, x0, [0, 4, 12, 30], seed + 7, torch.device("cuda", 0))
    ctx = twosd.SDContext(sp2, sto)
    ctx.compute_basis(x0, smps.mean_values(sto, positions))
    ctx.set_distributions(sto)
    tr = twosd.sdEpigraph(ctx, 1.0, 0.0)
    twosd.add_sampled_scenarios(tr, T, seed + 4)
    epi = twosd.sdEpigraph(ctx, 1.0, 0.0)
    twosd.add_sampled_scenarios(epi, N, seed)
    ctx.pool_refresh(tr, xs[-1], 0, T, P)
    for rnd in range(2):
        for it, xx in zip([0, 4, 12, 30], xs):
            ctx.pool_refresh(tr, xx, 0, T, P)
            ctx.pool_build_candidates(tr, xx, 0, T, 128, 160)
            obj, _, _, st = twosd.solve_batch(epi, xx, 0, N, want_pi=False)
            its, _ = ctx.last_lp_iters(N)
            tot = its.sum()
            srt = np.sort(its)[::-1]
            share = lambda q: srt[: int(q * N)].sum() / tot
            picks = ctx.last_pool_picks(N)
            if rnd == 1:
                print(f"x{it}: mean {its.mean():.2f} p50 {np.percentile(its, 50):.0f} p90 {np.percentile(its, 90):.0f} "
                      f"p99 {np.percentile(its, 99):.0f} max {its.max()} | zero-pivot {np.mean(its == 0):.3f} | "
                      f"pivot share of top 1% {share(0.01):.3f} top 10% {share(0.1):.3f} | "
                      f"primary-basis starts {np.mean(picks == 0):.3f} | LP {ctx.timings_us()[0] / 1e3:.2f} ms", flush=True)


if __name__ == "__main__":
    main()

"""Experiment: how the warm-start pool generalises across first-stage points.  Pivots per
scenario at SD candidate points for pools trained (a) at x_EV only, (b) at x_EV and other SD
iterates, (c) at the timed point itself (upper bound of what training can give)."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from sqlp_amd import smps, twosd
    import bench
    name = "storm"
    d = os.path.join(ROOT, "data", "smps", name)
    cor, tim, sto = smps.load_smps(d, name)
    sp2 = smps.get_smps_stage_template(cor, tim, 2)
    with open(os.path.join(ROOT, "tests", "golden", "ev_x.json")) as f:
        x_ev = np.array(json.load(f)[name]["x"])
    positions = list(sto.indep.keys())
    seed = 20250219
    its = [0, 2, 4, 6, 12, 20, 30]
    t0 = time.perf_counter()
    xs = dict(zip(its, bench.sd_points(cor, tim, sp2, sto, positions, x_ev, its, seed + 7, torch.device("cuda", 0))))
    print(f"trajectory {time.perf_counter() - t0:.1f}s", flush=True)
    P = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    N = 100000
    timed = [4, 12, 30]
    mode = sys.argv[2] if len(sys.argv) > 2 else "train"
    if mode == "refresh":
        ctx = twosd.SDContext(sp2, sto)
        ctx.compute_basis(x_ev, smps.mean_values(sto, positions))
        ctx.set_distributions(sto)
        tr = twosd.sdEpigraph(ctx, 1.0, 0.0)
        twosd.add_sampled_scenarios(tr, 4 * P, seed + 2)
        ctx.pool_build(tr, x_ev, 0, 4 * P, P)
        epi = twosd.sdEpigraph(ctx, 1.0, 0.0)
        twosd.add_sampled_scenarios(epi, N, seed)
        rt = twosd.sdEpigraph(ctx, 1.0, 0.0)
        twosd.add_sampled_scenarios(rt, 65536, seed + 5)
        for T, mp, l1 in [(16384, 1024, 0), (16384, 4096, 0), (16384, 4096, 128), (32768, 4096, 128), (65536, 8192, 128)]:
            for xt in timed:
                t1 = time.perf_counter()
                n = ctx.pool_refresh(rt, xs[xt], 0, T, mp)
                t_ref = time.perf_counter() - t1
                t1 = time.perf_counter()
                if l1:
                    ctx.pool_build_candidates(rt, xs[xt], 0, T, l1, 160)
                t_cand = time.perf_counter() - t1
                twosd.solve_batch(epi, xs[xt], 0, N, want_pi=False)
                piv, pmax = ctx.lp_stats()
                tm = ctx.timings_us()
                print(json.dumps({"refresh_T": T, "max_pool": mp, "level1": l1, "x": xt, "pool": n, "refresh_s": t_ref,
                                  "cand_s": t_cand,
                                  "refresh_ms": list(ctx.last_refresh_ms()), "pivots": piv / N, "pmax": pmax,
                                  "lp_ms": tm[0] / 1e3, "sel_ms": tm[4] / 1e3}), flush=True)
        return
    setups = {"ev_only": [0], "ev+2,6,20": [0, 2, 6, 20], "self": None}
    for label, train in setups.items():
        for xt in timed:
            ctx = twosd.SDContext(sp2, sto)
            ctx.compute_basis(x_ev, smps.mean_values(sto, positions))
            ctx.set_distributions(sto)
            tr_pts = train if train is not None else [xt]
            for j, xp in enumerate(tr_pts):
                tr = twosd.sdEpigraph(ctx, 1.0, 0.0)
                twosd.add_sampled_scenarios(tr, 4 * P // len(tr_pts), seed + 2 + 100 * j)
                ctx.pool_build(tr, xs[xp], 0, 4 * P // len(tr_pts), (P * (j + 1)) // len(tr_pts))
            epi = twosd.sdEpigraph(ctx, 1.0, 0.0)
            twosd.add_sampled_scenarios(epi, N, seed)
            twosd.solve_batch(epi, xs[xt], 0, N, want_pi=False)
            piv, pmax = ctx.lp_stats()
            tm = ctx.timings_us()
            # reference: primary basis only
            c0 = twosd.SDContext(sp2, sto)
            c0.compute_basis(x_ev, smps.mean_values(sto, positions))
            e0 = twosd.sdEpigraph(c0, 1.0, 0.0)
            c0.set_distributions(sto)
            twosd.add_sampled_scenarios(e0, 20000, seed)
            twosd.solve_batch(e0, xs[xt], 0, 20000, want_pi=False)
            p0, _ = c0.lp_stats()
            print(json.dumps({"train": label, "x": xt, "pool": ctx.pool_size(), "pivots": piv / N, "pmax": pmax,
                              "lp_ms": tm[0] / 1e3, "sel_ms": tm[4] / 1e3, "primary_pivots": p0 / 20000}), flush=True)
            ctx.close(); c0.close()


if __name__ == "__main__":
    main()

"""Pivot distribution of the pool-refresh training solves and the effect of a training pivot cap
(twosd_set_refresh_kcap) on the refresh time and on the pivots of the following main solve.

One wavefront solves one scenario, so a training launch of T scenarios on >= T wave slots lasts
as long as its slowest scenario.  Usage (GPU box):
    python tools/train_pivots.py [scenarios] [train] [pool] [caps...]
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    torch.cuda.init()
    import bench
    from sqlp_amd import smps, twosd
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 125000
    T = int(sys.argv[2]) if len(sys.argv) > 2 else 2048
    P = int(sys.argv[3]) if len(sys.argv) > 3 else 512
    # cap: an explicit pivot cap, "none" (kmax) or "auto" (4 x the last batch's mean, >= 32)
    caps = sys.argv[4:] or ["none", "auto", "48", "32", "24"]
    d = os.path.join(ROOT, "data", "smps", "storm")
    cor, tim, sto = smps.load_smps(d, "storm")
    sp2 = smps.get_smps_stage_template(cor, tim, 2)
    with open(os.path.join(ROOT, "tests", "golden", "ev_x.json")) as f:
        x0 = np.array(json.load(f)["storm"]["x"])
    positions = list(sto.indep.keys())
    xs = bench.sd_points(cor, tim, sp2, sto, positions, x0, [0, 4, 12, 30], 20250219 + 7, torch.device("cuda", 0))
    ctx = twosd.SDContext(sp2, sto)
    ctx.compute_basis(x0, smps.mean_values(sto, positions))
    ctx.set_distributions(sto)
    tr = twosd.sdEpigraph(ctx, 1.0, 0.0)
    twosd.add_sampled_scenarios(tr, T, 20250219 + 4)
    epi = twosd.sdEpigraph(ctx, 1.0, 0.0)
    twosd.add_sampled_scenarios(epi, N, 20250219)
    for cap in caps:
        ctx.set_refresh_kcap(-1)
        ctx.pool_refresh(tr, xs[-1], 0, T, P)
        ctx.set_refresh_kcap({"none": -1, "auto": 0}.get(cap) if cap in ("none", "auto") else int(cap))
        rows = []
        for xx in xs:
            t0 = time.perf_counter()
            ctx.pool_refresh(tr, xx, 0, T, P)
            if ctx.pool_size() > 128:
                ctx.pool_build_candidates(tr, xx, 0, T, 128, 160)
            t_ref = 1e3 * (time.perf_counter() - t0)
            its, st = ctx.last_lp_iters(T)
            parts = ctx.last_refresh_ms()
            ctx.invalidate_x()
            t1 = time.perf_counter()
            twosd.solve_push(epi, xx, 0, N, want_obj=False)
            t_main = 1e3 * (time.perf_counter() - t1)
            piv = ctx.lp_stats()[0] / N
            lp_ms = ctx.timings_us()[0] / 1e3
            rows.append((t_ref, parts[0], its, st, piv, lp_ms, t_main))
        print(f"cap {cap}: ", end="")
        for t_ref, t_train, its, st, piv, lp_ms, t_main in rows:
            ok = st == 0
            print(f"| refresh {t_ref:.2f} (train {t_train:.2f}) piv p50/p90/p99/max {np.percentile(its, 50):.0f}/"
                  f"{np.percentile(its, 90):.0f}/{np.percentile(its, 99):.0f}/{its.max()} dropped {int((~ok).sum())} "
                  f"-> main {piv:.2f} piv, LP {lp_ms:.2f} ms, push {t_main:.2f} ms ", end="")
        print(f"| mean refresh {np.mean([r[0] for r in rows]):.2f} main {np.mean([r[6] for r in rows]):.2f}", flush=True)


if __name__ == "__main__":
    main()

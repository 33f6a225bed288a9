"""Debug: the refresh sequence of bench.py with warmup 4 (first refresh at x_EV from the primary
basis, then x_4), printing the training statuses of each refresh (TWOSD_DEBUG) and the pool-start
outcome of solving x_4's training scenarios from the x_EV pool.
usage: TWOSD_DEBUG=1 python tools/debug_refresh_seq.py [N] [variant]"""
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
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 200000
    variant = sys.argv[2] if len(sys.argv) > 2 else "full"
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
    T, P = 16384, 4096
    tr = twosd.sdEpigraph(ctx, 1.0, 0.0)
    twosd.add_sampled_scenarios(tr, T, seed + 4)
    epi = twosd.sdEpigraph(ctx, 1.0, 0.0)
    twosd.add_sampled_scenarios(epi, N, seed)
    V = twosd.sdDualVertexSet(ctx)
    for step, xi in enumerate([0, 1, 2, 3]):
        xx = xs[xi]
        print(f"--- refresh at x{xi}", flush=True)
        ctx.pool_refresh(tr, xx, 0, T, P)
        if variant != "nocand" and ctx.pool_size() > 128:
            ctx.pool_build_candidates(tr, xx, 0, T, 128, 160)
        if variant == "nosolve":
            continue
        twosd.solve_push(epi, xx, 0, N, want_obj=False)
        ps, pm = ctx.lp_stats()
        print(f"x{xi}: main solve mean pivots {ps / N:.2f}, max {pm}, pool {ctx.pool_size()}", flush=True)
        if step == 0:
            # the next x's training scenarios solved from this pool (retry on)
            obj, _, _, st = twosd.solve_batch(tr, xs[1], 0, T, want_pi=False) if False else (None, None, None, None)
            o = np.zeros(T)
            stt = np.zeros(T, dtype=np.int32)
            import ctypes as C
            p = lambda a: a.ctypes.data_as(C.c_void_p)
            xx1 = np.ascontiguousarray(xs[1])
            rc = ctx.lib.twosd_solve_batch(ctx.h, tr.index, p(xx1), 0, T, p(o), None, None, p(stt))
            picks = ctx.last_pool_picks(T)
            ps, pm = ctx.lp_stats()
            print(f"  x1 training scenarios from the x0 pool: rc {rc}, statuses {np.bincount(stt, minlength=5)}, "
                  f"mean pivots {ps / T:.2f} max {pm}, retried from primary {(picks == 0).sum()}", flush=True)
            ctx.invalidate_x()


if __name__ == "__main__":
    main()

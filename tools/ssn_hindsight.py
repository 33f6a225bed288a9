"""Warm-start diagnosis for ssn (also storm at x_EV, item 3): is the pivot count limited by the pool's
CONTENT or by the device SELECTION?  At each bench x point of ssn (the bench protocol: the pool
refreshed at x from the training stream, 100k-scenario shard, 512-basis pool), a sample of the
shard's scenarios is solved
  * on the GPU from the device selection's pick (pivots per scenario, twosd_last_lp_iters),
  * by the C oracle (same pivot rules) from the primary basis, and
  * by the C oracle from EVERY pool basis: the least pivots over the pool per scenario is the
    best-in-hindsight start -- the floor any selection over this pool could reach -- and the
    pivots of the oracle from the device's pick (the same start as the GPU).
Also reported: the rank of the device pick among the pool bases by hindsight pivots, and the
pivots of the best start by the selection's own key (least primal infeasibility, the CPU pick).
Usage (GPU box): python tools/ssn_hindsight.py [sample] [threads] [x_points] [ssn|storm] > profiles/r05/ssn_hindsight.txt
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
    dev = torch.device("cuda", 0)
    import bench
    from oracle import cpu
    from sqlp_amd import smps, twosd
    S = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
    threads = int(sys.argv[2]) if len(sys.argv) > 2 else 16
    x_iters = [int(v) for v in (sys.argv[3] if len(sys.argv) > 3 else "0,4,12,30").split(",")]
    # instance and the bench's shard / pool for it (storm: 1M scenarios, 4096-basis pool)
    name = sys.argv[4] if len(sys.argv) > 4 else "ssn"
    N, POOL = {"ssn": (100_000, 512), "storm": (1_000_000, 4096)}[name]
    TRAIN = 4 * POOL
    seed = 20250219
    d = os.path.join(ROOT, "data", "smps", name)
    cor, tim, sto = smps.load_smps(d, name)
    sp2 = smps.get_smps_stage_template(cor, tim, 2)
    with open(os.path.join(ROOT, "tests", "golden", "ev_x.json")) as f:
        x0 = np.array(json.load(f)[name]["x"])
    positions = list(sto.indep.keys())
    xs = bench.sd_points(cor, tim, sp2, sto, positions, x0, x_iters, seed + 7, dev)
    ctx = twosd.SDContext(sp2, sto)
    ctx.compute_basis(x0, smps.mean_values(sto, positions))
    ctx.set_distributions(sto)
    epi = twosd.sdEpigraph(ctx, 1.0, 0.0)
    twosd.add_sampled_scenarios(epi, N, seed)
    rtr = twosd.sdEpigraph(ctx, 1.0, 0.0)
    twosd.add_sampled_scenarios(rtr, TRAIN, seed + 4)
    sam = twosd.sdEpigraph(ctx, 1.0, 0.0)
    vals = twosd.get_scenarios(epi, 0, S)
    twosd.add_scenarios(sam, vals)
    W, T = sp2.dense_W(), sp2.dense_T()
    lp = cpu.CpuLP(W, sp2.q, sp2.sense)
    rows = ctx.rows
    DR = vals - sp2.r[rows]
    head0 = ctx.get_basis()
    # the bench's warmup: two passes over the x points (pools trained from the previous x's pool)
    for xx in xs + xs:
        ctx.pool_refresh(rtr, xx, 0, TRAIN, POOL)
        ctx.pool_build_candidates(rtr, xx, 0, TRAIN, 128, 160)
        twosd.solve_batch(epi, xx, 0, N, want_pi=False)
    out = []
    for it, xx in zip(x_iters, xs):
        ctx.pool_refresh(rtr, xx, 0, TRAIN, POOL)
        ctx.pool_build_candidates(rtr, xx, 0, TRAIN, 128, 160)
        twosd.solve_batch(epi, xx, 0, N, want_pi=False)
        shard_piv = ctx.lp_stats()[0] / N
        _, _, _, st = twosd.solve_batch(sam, xx, 0, S, want_pi=False)
        gpu_it = ctx.last_lp_iters(S)[0]
        picks = ctx.last_pool_picks(S)
        P = ctx.pool_size()
        heads = np.stack([ctx.pool_get(p) for p in range(P)])
        base = sp2.r - T @ xx
        t0 = time.perf_counter()
        lp.set_basis(head0)
        _, _, _, st0, it0 = lp.solve_batch(rows, base, DR, kmax=2000, nthreads=threads)
        allit = np.full((P, S), 10 ** 6, dtype=np.int64)
        for p in range(P):
            if p % 128 == 0:
                print(f"x {it}: basis {p} of {P}", file=sys.stderr, flush=True)   # progress (a long storm pass)
            try:
                lp.set_basis(heads[p])
            except RuntimeError:
                continue
            _, _, _, stp, itp = lp.solve_batch(rows, base, DR, kmax=2000, nthreads=threads)
            allit[p] = np.where(stp == 0, itp, 10 ** 6)
        if P <= 1024:   # the oracle's pool keeps a dense inverse per basis (storm's 4096: 9 GB): skipped there
            lp.set_pool(heads)
            _, _, stc, itc, cpick = lp.solve_batch_pool(rows, base, DR, kmax=2000, nthreads=threads)
        else:
            stc, itc = np.zeros(1, np.int32), np.full(1, -1)
        t_cpu = time.perf_counter() - t0
        if os.environ.get("HINDSIGHT_DUMP"):   # the per-(basis, scenario) pivots for an offline study of selection keys
            np.savez_compressed(f"{os.environ['HINDSIGHT_DUMP']}_{name}_x{it}.npz", allit=allit.astype(np.int32), heads=heads,
                                picks=picks, gpu_it=gpu_it, vals=vals, x=xx, rows=rows, it0=it0)
        best = allit.min(0)
        at_pick = allit[picks, np.arange(S)]
        rank = (allit < at_pick[None, :]).sum(0)      # pool bases strictly better than the pick
        ok = (st == 0) & (best < 10 ** 6)
        row = {"x_iteration": it, "pool": int(P), "sample": S, "shard_pivots_mean": round(float(shard_piv), 2),
               "gpu_pick_pivots_mean": round(float(gpu_it[ok].mean()), 2),
               "oracle_at_gpu_pick_mean": round(float(at_pick[ok].mean()), 2),
               "hindsight_best_mean": round(float(best[ok].mean()), 2),
               "hindsight_best_p50_p90_max": [int(np.percentile(best[ok], 50)), int(np.percentile(best[ok], 90)), int(best[ok].max())],
               "primary_basis_mean": round(float(it0[st0 == 0].mean()), 2),
               "oracle_level1_pick_mean": round(float(itc[stc == 0].mean()), 2),
               "pick_rank_mean": round(float(rank[ok].mean()), 1),
               "pick_is_hindsight_best": round(float((at_pick[ok] == best[ok]).mean()), 3),
               "scenarios_whose_best_start_is_primary": round(float((allit[0][ok] == best[ok]).mean()), 3),
               "distinct_best_bases": int(len(np.unique(allit.argmin(0)[ok]))),
               "gpu_iter_over_200": int((gpu_it > 200).sum()), "cpu_s": round(t_cpu, 1)}
        out.append(row)
        print(json.dumps(row), flush=True)
    print(json.dumps({"summary": "ssn warm-start diagnosis", "rows": out}), flush=True)


if __name__ == "__main__":
    main()

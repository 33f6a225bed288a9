"""Per-rank step of the N-GPU bench (strong scaling of the storm 1M batch), emulated on ONE GPU:
G contexts in one process, one per emulated rank, each with its own 1/G scenario shard and its
1/G slice of the refresh training scenarios.  Every phase of a rank runs alone on the GPU, in
sequence: the distributed refresh (twosd_refresh_train, the global selection, the local
composition, the assembly from the gathered packs, the candidate picks), then solve_push and
the cut over the rank's shard.  The all-gathers travel by device copies here; their xGMI time is
estimated as bytes / (link_gbs) per peer pack (each GPU receives the G-1 other packs over its G-1
point-to-point links in parallel) and added -- it is the one number not measured.

Per-rank step = the rank's own phases + the exchange estimate; reported per x point and as the
max over ranks, next to N = 1 (one context holding everything, the bench's single-GPU step).
Usage (GPU box): python tools/shard_emulate.py [G] [scenarios] [steps] [pool] [training scenarios] [warmup]
(the bench protocol: `warmup` untimed steps cycling over the x points, then `steps` reported ones;
every refresh trains from the current pool, so revisited x points get better pools, as in bench.py)
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

LINK_GBS = 153.0 * 0.5       # xGMI link, half of the per-link figure (RCCL efficiency assumed)
COLLECTIVE_MS = 0.05         # latency of one small RCCL collective + its host synchronisation (assumed)
REFRESH_COLLECTIVES = 6      # collectives of one distributed refresh (sqlp_amd.dist.refresh_sharded)
STEP_COLLECTIVES = 4         # per step besides the refresh: 2 for the vertex all-gather, 2 for the cut partials
                             # (sums + incumbent objective + the vertex-set check, then the histogram)


def main():
    import torch
    torch.cuda.init()
    dev = torch.device("cuda", 0)
    import bench
    from sqlp_amd import dist as sdist
    from sqlp_amd import smps, twosd
    G = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    N = int(sys.argv[2]) if len(sys.argv) > 2 else 1_000_000
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 8
    POOL = int(sys.argv[4]) if len(sys.argv) > 4 else 4096
    TRAIN = int(sys.argv[5]) if len(sys.argv) > 5 else 4 * POOL
    WARMUP = int(sys.argv[6]) if len(sys.argv) > 6 else 5
    seed = 20250219
    L1, NC, NV = 128, 160, 4096
    d = os.path.join(ROOT, "data", "smps", "storm")
    cor, tim, sto = smps.load_smps(d, "storm")
    sp2 = smps.get_smps_stage_template(cor, tim, 2)
    with open(os.path.join(ROOT, "tests", "golden", "ev_x.json")) as f:
        x0 = np.array(json.load(f)["storm"]["x"])
    positions = list(sto.indep.keys())
    xs = bench.sd_points(cor, tim, sp2, sto, positions, x0, [0, 4, 12, 30], seed + 7, dev)
    ranks = []
    for r in range(G):
        ctx = twosd.SDContext(sp2, sto)
        ctx.compute_basis(x0, smps.mean_values(sto, positions))
        ctx.set_distributions(sto)
        lo, hi = sdist.shard_range(N, r, G)
        epi = twosd.sdEpigraph(ctx, 1.0, 0.0)
        twosd.add_sampled_scenarios(epi, hi - lo, seed, first_index=lo)
        tlo, thi = sdist.shard_range(TRAIN, r, G)
        tr = twosd.sdEpigraph(ctx, 1.0, 0.0)
        twosd.add_sampled_scenarios(tr, thi - tlo, seed + 4, first_index=tlo)
        V = twosd.sdDualVertexSet(ctx)
        ranks.append(dict(ctx=ctx, epi=epi, tr=tr, n=hi - lo, nt=thi - tlo, V=V))
    # |V| pool (identical on every rank): duals of stream seed + 1
    src = twosd.sdEpigraph(ranks[0]["ctx"], 1.0, 0.0)
    twosd.add_sampled_scenarios(src, 1 << 18, seed + 1)
    V0 = twosd.sdDualVertexSet(ranks[0]["ctx"])
    at = 0
    while len(V0) < NV and at < (1 << 18):     # as bench.py
        _, _, pis, st = twosd.solve_batch(src, x0, at, 16384, want_pi=True)
        V0.push_batch(pis[st == 0])
        at += 16384
    V0.truncate(min(NV, len(V0)))
    Vm = V0.matrix()
    for rk in ranks[1:]:
        rk["V"].push_batch(Vm)
    nv = len(V0)

    def refresh(xx):
        """the distributed refresh, phase by phase per rank; returns per-rank ms and pack bytes"""
        ms = [dict() for _ in range(G)]
        lists = []
        # one training cap for all ranks (sqlp_amd.dist.refresh_training_cap: 3 x the mean pivots
        # of every rank's last large batch, at least 32)
        ps = sum(rk["ctx"].refresh_cap_stats()[0] for rk in ranks)
        pn = sum(rk["ctx"].refresh_cap_stats()[1] for rk in ranks)
        cap = ranks[0]["ctx"].training_cap(ps, pn)     # the native rule (twosd_training_cap)
        nopt = []
        for r, rk in enumerate(ranks):
            t = time.perf_counter()
            k, c, f, lo_, hi_, no = rk["ctx"].refresh_train_ex(rk["tr"], xx, 0, rk["nt"], cap)
            ms[r]["train"] = 1e3 * (time.perf_counter() - t)
            lists.append((k, c, f, lo_, hi_))
            nopt.append(no)
        if cap > 0 and 2 * sum(nopt) < sum(rk["nt"] for rk in ranks):    # the global uncapped retry
            lists = []
            for r, rk in enumerate(ranks):
                t = time.perf_counter()
                k, c, f, lo_, hi_, no = rk["ctx"].refresh_train_ex(rk["tr"], xx, 0, rk["nt"], 0)
                ms[r]["train"] += 1e3 * (time.perf_counter() - t)
                lists.append((k, c, f, lo_, hi_))
        t = time.perf_counter()
        kk = np.concatenate([l[0] for l in lists])
        cc = np.concatenate([l[1] for l in lists]).astype(np.int64)
        ff = np.concatenate([l[2] for l in lists]).astype(np.int64)
        rk_of = np.concatenate([np.full(len(l[0]), r) for r, l in enumerate(lists)])
        owner, orep = sdist.select_refresh_bases(kk, cc, ff, rk_of, POOL)
        box_lo = np.min([l[3] for l in lists], axis=0)
        box_hi = np.max([l[4] for l in lists], axis=0)
        pos = sdist.pack_positions(owner, G)
        t_sel = 1e3 * (time.perf_counter() - t)
        nbytes = []
        for r, rk in enumerate(ranks):
            ms[r]["select"] = t_sel
            t = time.perf_counter()
            nbytes.append(rk["ctx"].refresh_build_local(orep[owner == r]))
            ms[r]["build"] = 1e3 * (time.perf_counter() - t)
        stride = (max(nbytes) + 255) // 256 * 256
        out = torch.empty(G * stride, dtype=torch.uint8, device=dev)
        torch.cuda.synchronize()
        for r, rk in enumerate(ranks):
            rk["ctx"].refresh_pack(out[r * stride:].data_ptr())
        for r, rk in enumerate(ranks):
            t = time.perf_counter()
            rk["ctx"].refresh_assemble(G, out.data_ptr(), stride, pos, box_lo, box_hi)
            ms[r]["assemble"] = 1e3 * (time.perf_counter() - t)
        picks = []
        for r, rk in enumerate(ranks):
            t = time.perf_counter()
            picks.append(rk["ctx"].pool_candidate_picks(rk["tr"], xx, 0, rk["nt"], L1))
            ms[r]["picks"] = 1e3 * (time.perf_counter() - t)
        p1 = np.concatenate([p[0] for p in picks])
        pf = np.concatenate([p[1] for p in picks])
        for r, rk in enumerate(ranks):
            t = time.perf_counter()
            rk["ctx"].pool_set_candidates(L1, NC, p1, pf)
            ms[r]["cand_lists"] = 1e3 * (time.perf_counter() - t)
            # exchanges: the packs by bandwidth (each GPU receives the G - 1 other packs over its
            # G - 1 links in parallel) plus a fixed latency per collective and host synchronisation
            # (sqlp_amd.dist.refresh_sharded: cap all-reduce, header, payload, pack size, packs, picks)
            ms[r]["xgmi_est"] = (1e3 * (max(nbytes[q] for q in range(G) if q != r) if G > 1 else 0) / (LINK_GBS * 1e9) +
                                 REFRESH_COLLECTIVES * COLLECTIVE_MS)
        return ms, nbytes, int(ranks[0]["ctx"].pool_size())

    def solve_cut(rk, xx):
        t = time.perf_counter()      # the refresh prepared x (its candidate picks): no invalidate
        twosd.solve_push(rk["epi"], xx, 0, rk["n"], want_obj=False)
        tm = rk["ctx"].timings_us()
        rk["V"].truncate(nv)
        piv = rk["ctx"].lp_stats()[0] / rk["n"]
        twosd.build_sasa_cut(rk["epi"], xx, rk["V"], 0.0)
        tc = rk["ctx"].timings_us()
        # device phases of the solve + cut (HIP events): selection, LP, dedup, cut
        rk["phases"] = {"sel": tm[4] / 1e3, "lp": tm[0] / 1e3, "dedup": tm[1] / 1e3, "cut": (tc[2] + tc[3]) / 1e3}
        return 1e3 * (time.perf_counter() - t), piv

    refresh(xs[-1])       # the pool at the last x point
    for i in range(WARMUP):   # untimed steps ending at the last x point (bench.py's warmup)
        xx = xs[(i - WARMUP) % len(xs)]
        refresh(xx)
        for rk in ranks:
            solve_cut(rk, xx)
    rows = []
    for i in range(steps):
        xx = xs[i % len(xs)]
        ms, nbytes, P = refresh(xx)
        per = []
        for r, rk in enumerate(ranks):
            t_sc, piv = solve_cut(rk, xx)
            ms[r]["solve_cut"] = t_sc
            ms[r]["solve_cut_device"] = {k: round(v, 2) for k, v in rk["phases"].items()}
            ms[r]["step_collectives_est"] = STEP_COLLECTIVES * COLLECTIVE_MS
            per.append((sum(v for v in ms[r].values() if not isinstance(v, dict)), piv))
        worst = max(range(G), key=lambda r: per[r][0])
        rows.append((i % len(xs), per[worst][0], np.mean([p[0] for p in per]), np.mean([p[1] for p in per]), P,
                     {k: (round(v, 2) if not isinstance(v, dict) else v) for k, v in ms[worst].items()}, max(nbytes)))
        print(f"x{rows[-1][0]}: per-rank step max {rows[-1][1]:.2f} ms (mean {rows[-1][2]:.2f}), pivots {rows[-1][3]:.2f}, "
              f"pool {P}, pack {max(nbytes) / 1e6:.1f} MB, slowest rank {rows[-1][5]}", flush=True)
    step_ms = float(np.mean([r[1] for r in rows]))
    print(json.dumps({"G": G, "scenarios": N, "pool": POOL, "train": TRAIN, "warmup": WARMUP, "steps": steps, "per_rank_step_ms": step_ms,
                      "subproblems_per_s_projected": N / (step_ms * 1e-3),
                      "note": f"emulated on one GPU; xGMI all-gather estimated at {LINK_GBS} GB/s per link, "
                              f"{COLLECTIVE_MS} ms per collective ({REFRESH_COLLECTIVES} per refresh, "
                              f"{STEP_COLLECTIVES} per step besides)"}), flush=True)


if __name__ == "__main__":
    main()

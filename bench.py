#!/usr/bin/env python3
"""bench.py -- TwoSD scenario-subproblem + cut-generation hot path on MI355X.

Metric (BASELINE.json): stage-2 subproblems/sec + cut-gen HBM GB/s on STORM.
One step = one pass of the hot path over the (sharded) scenario batch at a first-stage x:
  1. solve_problem! for every scenario of the shard (GPU dual simplex, LP kernel),
  2. push! of every dual into the dual vertex set (device dedup by dual keys), then rollback
     of the set to the fixed |V| pool so every step sees the same set (fixed |V|),
  3. build_sasa_cut over the same scenarios with the |V| pool (MFMA argmax + cut),
     RCCL all-reduce of the cut partials when N > 1, plus the SD-sized vertex all-gather
     (2 new vertices per epigraph per step, as sd_iteration! adds).
The timed steps cycle over X first-stage points: the EV solution (where the warm-start pool
and its candidate lists were trained) and X-1 candidate points of an SD run on the same
instance (master QP + GPU hot path, sqlp_amd/master.py), so the pool is timed at points it
was not trained at.  Pivots and ms are reported per point.
value = scenarios processed by all ranks / max-over-ranks time of the K timed steps.

Workload: storm (data/smps/storm, reference spInput), 1,000,000 i.i.d. synthetic scenarios
from storm.sto drawn on the device, |V| = 4096 real LP duals.  Strong scaling: the 1M
scenarios are split over the ranks.  After the timed region: a parity spot check of 4096
scenarios per x point against the C oracle (LP objectives, cut alpha/beta) and the CPU
baseline (C port, primary-basis and pooled warm starts).

Run:  python bench.py [--gpus N --steps K --warmup W]
      python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PEAK_HBM_GBS = 8000.0        # MI355X HBM3E spec (MI355X_MICROARCH.md)
PEAK_FP64_TFS = 78.6         # MI355X fp64 (vector == matrix on gfx950), spec
PEAK_F32_MFMA_TFS = 157.3    # MI355X fp32-input MFMA (v_mfma_f32_16x16x4_f32), spec (MI355X_MICROARCH.md)
CHUNK = 1 << 16


def chunked_values(sto, positions, lo, hi, seed):
    """Scenario values [lo, hi) of the global stream: chunk c is drawn with seed (seed, c)."""
    from sqlp_amd import smps
    out = np.empty((hi - lo, len(positions)))
    c0, c1 = lo // CHUNK, (hi - 1) // CHUNK
    for c in range(c0, c1 + 1):
        a, b = c * CHUNK, (c + 1) * CHUNK
        vals = smps.sample_values(sto, CHUNK, np.random.default_rng([seed, c]), positions)
        s, e = max(a, lo), min(b, hi)
        out[s - lo:e - lo] = vals[s - a:e - a]
    return out


def importance_values(sto, positions, lo, hi, seed, scale):
    """Scenarios [lo, hi) of an importance-sampled stream (config C5): every NORMAL element
    drawn from N(mu, (scale sigma)^2), other elements from their own distribution; weight =
    likelihood ratio target / proposal (per-chunk seeds: sharding-invariant)."""
    from sqlp_amd import smps
    k = len(positions)
    vals = chunked_values(sto, positions, lo, hi, seed)
    out_w = np.ones(hi - lo)
    c0, c1 = lo // CHUNK, (hi - 1) // CHUNK
    for j, pos in enumerate(positions):
        dist = sto.indep[pos]
        if dist[0] != "NORMAL":
            continue
        mu, sd = dist[1], np.sqrt(dist[2])     # NORMAL(mean, variance), smps_sto.jl:122-125
        z = np.empty(hi - lo)
        for c in range(c0, c1 + 1):
            a, b = c * CHUNK, (c + 1) * CHUNK
            zz = np.random.default_rng([seed, c, j, 7]).standard_normal(CHUNK)
            s_, e_ = max(a, lo), min(b, hi)
            z[s_ - lo:e_ - lo] = zz[s_ - a:e_ - a]
        v = mu + scale * sd * z
        vals[:, j] = v
        out_w *= scale * np.exp(-0.5 * z * z * (scale * scale) + 0.5 * z * z)
    del k
    return vals, out_w


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=8)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--instance", default="storm")
    ap.add_argument("--scenarios", type=int, default=1_000_000)
    ap.add_argument("--vertices", type=int, default=4096)
    ap.add_argument("--tie-rel", type=float, default=0.0,
                    help="argmax tie rule: 0 = the reference's strict '>' (subprob.jl:156, first maximum); > 0 the "
                         "build's near-tie rule (DESIGN.md §3)")
    ap.add_argument("--seed", type=int, default=20250219)
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="wall budget of the CPU baseline sample")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-dedup", action="store_true")
    ap.add_argument("--x-points", default="0,4,12,30",
                    help="first-stage points the timed steps cycle over: 0 = the EV solution (pool training "
                         "point), i > 0 = the candidate of SD iteration i (storm master + GPU hot path)")
    ap.add_argument("--spot", type=int, default=4096, help="parity spot-check scenarios per x point (0: off)")
    ap.add_argument("--trajectory", type=int, default=20,
                    help="K > 0: after the timed cycle, time K more steps at K DISTINCT consecutive SD candidates "
                         "(iterations last+1 .. last+K of the same SD run, no revisits), reported beside the cycle")
    ap.add_argument("--refresh", type=int, default=1,
                    help="1: a step at an x other than the pool's rebuilds the pool there (twosd_pool_refresh + "
                         "candidate lists, inside the timed step); 0: keep the x_EV pool for every x")
    ap.add_argument("--refresh-train", type=int, default=0,
                    help="training scenarios of a pool refresh (0: 4 x the refresh pool)")
    ap.add_argument("--refresh-cand-train", type=int, default=0,
                    help="training scenarios whose flat picks build the two-level candidate lists after a refresh "
                         "(0: the --refresh-train ones; more extends the same stream)")
    ap.add_argument("--refresh-pool", type=int, default=0,
                    help="pool size after a refresh (0: 4096 per 1M scenarios of the refreshing ranks, at least 512)")
    ap.add_argument("--refresh-dist", type=int, default=1,
                    help="N > 1: 1 = the ranks split the refresh (each trains on 1/N of the training scenarios and "
                         "composes its share of the pool, packs all-gathered: sqlp_amd.dist.refresh_sharded); "
                         "0 = every rank refreshes alone from all training scenarios with a pool sized by its shard")
    ap.add_argument("--refresh-passes", type=int, default=1,
                    help="refreshes per new x: 2 = refresh again from the pool the first pass built (its training "
                         "solves start closer), both inside the timed step")
    ap.add_argument("--cpu-pool", type=int, default=128, help="bases of the pooled CPU baseline (0: off)")
    ap.add_argument("--pool", type=int, default=0,
                    help="warm-start basis pool size (1 = primary basis only; 0 = by the per-rank shard: "
                         "32768 from 500k scenarios per GPU, else 16384)")
    ap.add_argument("--pool-train", type=int, default=0, help="training scenarios of the pool build (0 = 4 x pool)")
    ap.add_argument("--pool-level1", type=int, default=128,
                    help="two-level warm-start selection: level 1 over the first L pool bases (0: flat)")
    ap.add_argument("--pool-cands", type=int, default=160, help="level-2 candidate bases per level-1 basis")
    ap.add_argument("--cand-train", type=int, default=262144, help="training scenarios of the candidate lists")
    ap.add_argument("--sampler", choices=["device", "host"], default="device",
                    help="scenario draws: on-device Philox4x32-10 sampler (twosd_add_sampled_scenarios) or numpy PCG64")
    ap.add_argument("--epigraphs", type=int, default=1,
                    help="E > 1: config C5 shape -- E epigraphs (objective weight 1/E), N/E scenarios each, "
                         "one shared vertex set, one cut per epigraph per step")
    ap.add_argument("--importance-scale", type=float, default=0.0,
                    help="s > 0: importance sampling of NORMAL elements from N(mu, (s sigma)^2) with "
                         "likelihood-ratio weights passed as add_scenario! weights (host draws)")
    args = ap.parse_args()

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    # TWOSD_BENCH_SHARED_GPU=1 (rehearsal only): every rank on cuda:0 with gloo collectives,
    # so the N > 1 path can be exercised on a one-GPU box; the real run is one rank per GPU
    # over RCCL
    shared = os.environ.get("TWOSD_BENCH_SHARED_GPU") == "1"
    device = torch.device("cuda", 0 if shared else local_rank)
    torch.cuda.set_device(device)
    if world > 1:
        import torch.distributed as dist
        if shared:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=device)
    from sqlp_amd import smps, twosd
    from sqlp_amd import dist as sdist

    name = args.instance
    d = os.path.join(ROOT, "data", "smps", name)
    cor, tim, sto = smps.load_smps(d, name)
    sp2 = smps.get_smps_stage_template(cor, tim, 2)
    with open(os.path.join(ROOT, "tests", "golden", "ev_x.json")) as f:
        x = np.array(json.load(f)[name]["x"])
    positions = list(sto.indep.keys())
    # first-stage points of the timed steps: x_EV and SD candidates (identical on every rank)
    t_traj = time.perf_counter()
    x_iters = sorted({int(v) for v in args.x_points.split(",")})
    traj_iters = list(range(max(x_iters) + 1, max(x_iters) + 1 + max(0, args.trajectory)))
    xs = sd_points(cor, tim, sp2, sto, positions, x, x_iters + traj_iters, args.seed + 7, device)
    if world > 1:
        t = torch.tensor(np.stack(xs), dtype=torch.float64, device=device)
        torch.distributed.broadcast(t, 0)
        xs = [row for row in t.cpu().numpy()]
    xs, xs_traj = xs[:len(x_iters)], xs[len(x_iters):]
    t_traj = time.perf_counter() - t_traj
    ctx = twosd.SDContext(sp2, sto, device=device.index)
    ctx.compute_basis(x, smps.mean_values(sto, positions))

    if args.sampler == "device":
        ctx.set_distributions(sto)

    def scenarios(epi_, lo_, hi_, seed_):
        """Scenarios [lo_, hi_) of the global stream `seed_` appended to epi_ (sharding-invariant)."""
        if args.sampler == "device":
            twosd.add_sampled_scenarios(epi_, hi_ - lo_, seed_, first_index=lo_)
        else:
            twosd.add_scenarios(epi_, chunked_values(sto, positions, lo_, hi_, seed_))

    # warm-start basis pool (setup, untimed like compute_basis): optimal bases of independent
    # training scenarios of the same distribution (seed + 2, identical on every rank)
    # pool size by the per-rank shard (profiles/r01/configs/pool_sweep7.jsonl): a larger pool
    # saves pivots but its per-x preparation (x_B, selection stream) is a fixed cost per step
    # and its B^-1 data competes for L2, so small shards (the N > 1 steps) prefer 16384
    # with the per-x refresh on, the timed steps never use the setup pool (the warmup's refresh
    # replaces it), so only the primary basis is installed
    if args.pool <= 0:
        args.pool = 1 if args.refresh else (32768 if args.scenarios // max(1, args.epigraphs) // world >= 500_000
                                            else 16384)
    if args.pool_train <= 0:
        args.pool_train = 4 * args.pool
    t_pool = time.perf_counter()
    if args.pool > 1:
        tr = twosd.sdEpigraph(ctx, 1.0, 0.0)
        scenarios(tr, 0, args.pool_train, args.seed + 2)
        ctx.pool_build(tr, x, 0, args.pool_train, args.pool)
    pool_size = ctx.pool_size()
    if args.pool_level1 > 0 and pool_size > args.pool_level1:
        ct = twosd.sdEpigraph(ctx, 1.0, 0.0)
        scenarios(ct, 0, args.cand_train, args.seed + 3)
        ctx.pool_build_candidates(ct, x, 0, args.cand_train, args.pool_level1, args.pool_cands)
    t_pool = time.perf_counter() - t_pool

    N = args.scenarios
    E = max(1, args.epigraphs)
    if N % E:
        raise SystemExit("--scenarios must be a multiple of --epigraphs")
    NE = N // E                    # scenarios per epigraph (global)
    lo, hi = sdist.shard_range(NE, rank, world)
    n_local = hi - lo              # per epigraph on this rank
    t_gen = time.perf_counter()
    epis, total_weights = [], []
    for e in range(E):
        epi_e = twosd.sdEpigraph(ctx, 1.0 / E, 0.0)
        if args.importance_scale > 0:
            vals, w = importance_values(sto, positions, lo, hi, args.seed + 101 * (e + 1), args.importance_scale)
            twosd.add_scenarios(epi_e, vals, w)
            # global total weight: sum over the ranks' shards (host all-reduce of one number)
            tw = float(w.sum())
            if world > 1:
                t = torch.tensor([tw], dtype=torch.float64, device=device)
                torch.distributed.all_reduce(t)
                tw = float(t.item())
            total_weights.append(tw)
        else:
            scenarios(epi_e, lo, hi, args.seed + 101 * e)
            total_weights.append(float(NE))   # all weights 1.0 (sd_iteration! uses 1.0, algorithm.jl:46)
        epis.append(epi_e)
    epi = epis[0]
    t_gen = time.perf_counter() - t_gen

    # |V| pool: duals of the first scenarios of the global stream seed + 1 (identical on every rank)
    V = twosd.sdDualVertexSet(ctx)
    src = twosd.sdEpigraph(ctx, 1.0, 0.0)
    scenarios(src, 0, 1 << 18, args.seed + 1)
    at = 0
    piv_primary = [0, 0]   # pivots / scenarios of these solves: the instance's LP cost from the primary basis
    while len(V) < args.vertices and at < (1 << 18):
        _, _, pis, st = twosd.solve_batch(src, x, at, 16384, want_pi=True)
        V.push_batch(pis[st == 0])
        piv_primary[0] += ctx.lp_stats()[0]
        piv_primary[1] += 16384
        at += 16384
    piv_primary = piv_primary[0] / max(piv_primary[1], 1)
    if len(V) > args.vertices:
        V.truncate(args.vertices)
    nv = len(V)

    X = len(xs)
    # refresh size by the per-rank shard: the refresh is a fixed cost per step (training solves,
    # B^-1 composition, upload grow with the pool), so a smaller shard takes a smaller pool
    # a distributed refresh builds one pool for all ranks, so it is sized by the whole batch
    dist_refresh = world > 1 and args.refresh_dist == 1
    if dist_refresh and args.refresh_cand_train > 0:
        # the distributed refresh builds the candidate lists from each rank's slice of the
        # refresh-training scenarios (sqlp_amd.dist.refresh_sharded): the knob would be ignored
        raise SystemExit("--refresh-cand-train applies to the single-rank refresh only (use --refresh-dist 0)")
    # pool size by the shard: 4096 per 1M scenarios on one rank, at least 512; the distributed
    # refresh builds four times that (at least 1024): its training and composition are split over
    # the ranks (profiles/r04/n8/shard_emulate_pool*.txt: at N = 8 with the bench warmup, pools of
    # 1024 / 1536 / 2048 / 3072 / 4096 bases give 18.7 / 18.3 / 18.4 / 20.3 / 22.1 ms per rank)
    # instances whose LPs are long from the primary basis (ssn: ~39 pivots, ~20 etas traversed per
    # pivot) take at least 2048 bases: the training solves cost more, the main solve saves more
    # (ssn 100k on the driver protocol, profiles/r06/ab_ssn_pool.txt: 512 / 1024 / 2048 / 4096 bases
    # -> 88.1 / 88.2 / 83.4 / 85.1 ms per step)
    if args.refresh_pool <= 0:
        scope = 4 * n_local * E if dist_refresh else n_local * E
        floor = 2048 if piv_primary > 16 else (1024 if dist_refresh else 512)
        args.refresh_pool = max(floor, min(4096, int(4096 * scope / 1_000_000) // 256 * 256))
    if args.refresh_train <= 0:
        args.refresh_train = 4 * args.refresh_pool
    # pool refresh training scenarios (stream seed + 4; every rank holds all of them, or with
    # the distributed refresh its contiguous slice)
    rtr = None
    t_lo, t_hi = sdist.shard_range(args.refresh_train, rank, world) if dist_refresh else (0, args.refresh_train)
    # the candidate lists may take more training scenarios than the pool (single-rank refresh): the
    # same stream, extended
    if not dist_refresh and args.refresh_cand_train > args.refresh_train:
        t_hi = args.refresh_cand_train
    if args.refresh:
        rtr = twosd.sdEpigraph(ctx, 1.0, 0.0)
        scenarios(rtr, t_lo, t_hi, args.seed + 4)
    # the pool is not at any x point yet: the first step at every x pays its refresh (the
    # setup pool, if any, was built at x_EV from other training scenarios)
    pool_at = {"x": None}

    def refresh(xx):
        """Per-x warm-start pool: rebuilt from the training scenarios' optimal bases at xx
        (timed as part of the step), two-level selection lists from the same scenarios."""
        if rtr is None or (pool_at["x"] is not None and np.array_equal(pool_at["x"], xx)):
            return 0.0
        t0 = time.perf_counter()
        if dist_refresh:
            for _ in range(max(1, args.refresh_passes)):
                _, ms = sdist.refresh_sharded(ctx, rtr, xx, 0, t_hi - t_lo, args.refresh_pool, args.pool_level1,
                                              args.pool_cands, device)
            pool_at["x"] = xx.copy()
            pool_at["last_ms"] = ms
            return time.perf_counter() - t0
        for _ in range(max(1, args.refresh_passes)):
            ctx.pool_refresh(rtr, xx, 0, args.refresh_train, args.refresh_pool)
        t1 = time.perf_counter()
        if args.pool_level1 > 0 and ctx.pool_size() > args.pool_level1:
            nct = args.refresh_train if args.refresh_cand_train <= 0 else args.refresh_cand_train
            ctx.pool_build_candidates(rtr, xx, 0, nct, args.pool_level1, args.pool_cands)
        pool_at["x"] = xx.copy()
        # ms: training solves (with eta files), basis keys + selection, pool build (device:
        # B^-1 FTRAN + pool arrays; host path: composition), host upload (host path only),
        # refresh total, two-level candidate lists
        ms = list(ctx.last_refresh_ms()) + [1e3 * (time.perf_counter() - t1)]
        pool_at["last_ms"] = dict(zip(("train", "keys", "build", "host_upload", "total", "candidates"), ms))
        return time.perf_counter() - t0

    step_obj = {"value": None}   # incumbent objective of the last step
    heads_at = {}    # first pool bases at each x point (the pooled CPU baseline starts from the same bases)

    def step(xx, rec=None, per_x_stats=True):
        t_ref = refresh(xx)
        if rec and per_x_stats:
            per_x[cur["xi"]]["refresh"] += t_ref
            if t_ref > 0:
                per_x[cur["xi"]]["refresh_parts"] = {k_: round(v, 2) for k_, v in pool_at["last_ms"].items()}
            if cur["xi"] not in heads_at and not args.no_cpu and rank == 0:
                heads_at[cur["xi"]] = np.stack([ctx.pool_get(p) for p in range(min(args.cpu_pool, ctx.pool_size()))])
        # every pass pays its per-x setup (x_B of the pool, selection data): a step that refreshed
        # paid it inside the refresh (the candidate lists select at this x, with this pool)
        if t_ref == 0.0:
            ctx.invalidate_x()
        alpha = 0.0
        objective = 0.0
        for epi_e, tw in zip(epis, total_weights):
            if args.no_dedup:
                twosd.solve_batch(epi_e, xx, 0, n_local, want_pi=False)
            else:
                twosd.solve_push(epi_e, xx, 0, n_local, want_obj=False)
                if world > 1:
                    # exchange (2) at the SD volume: two new vertices per epigraph (the candidate
                    # and incumbent duals of sd_iteration!, algorithm.jl:46-54) all-gathered
                    # and pushed in (rank, index) order on every rank
                    new = V.matrix(nv, min(2, len(V) - nv)) if len(V) > nv else np.zeros((0, m))
                    V.truncate(nv)
                    sdist.push_sharded(V, new)
                V.truncate(nv)
            # incumbent objective at xx: sum_s w_s obj_s / sum_s w_s of the epigraph's scenarios (device
            # reduction of the solve; across ranks all-reduced together with the cut partials)
            obj_sums = ctx.last_objective()
            if world == 1:
                alpha += twosd.build_sasa_cut(epi_e, xx, V, args.tie_rel).alpha / E
            else:
                a_, _, obj_sums = sdist.build_cut_sharded(ctx, epi_e, xx, tw, args.tie_rel, device, extra=obj_sums)
                alpha += a_ / E
            objective += obj_sums[0] / obj_sums[1] / E
            if rec:
                rec()      # per-epigraph kernel timings (HIP events of the last calls)
        step_obj["value"] = objective
        return alpha

    def barrier():
        torch.cuda.synchronize(device)
        if world > 1:
            torch.distributed.barrier()
        torch.cuda.synchronize(device)

    m = sp2.shape[0]
    # warmup steps cycle over the x points so that the last one is at xs[-1]: the first timed
    # step (at xs[0]) then pays its refresh like every later one
    for i in range(args.warmup):
        step(xs[(i - args.warmup) % X])
    barrier()
    acc = {"lp": 0.0, "dd": 0.0, "cut": 0.0, "fin": 0.0, "sel": 0.0, "flops": 0.0, "piv": 0, "pmax": 0, "eta": 0, "retries": 0}
    per_x = [{"piv": 0, "n": 0, "lp": 0.0, "wall": 0.0, "steps": 0, "alpha": None, "refresh": 0.0, "eta": 0, "reps": 0, "full": 0}
             for _ in xs]
    cur = {"xi": 0, "piv": 0, "lp": 0.0}

    def record():
        tm = ctx.timings_us()
        acc["lp"] += tm[0]; acc["dd"] += tm[1]; acc["cut"] += tm[2]; acc["fin"] += tm[3]; acc["sel"] += tm[4]
        acc["flops"] += ctx.lp_flops()
        eta, retries = ctx.lp_counts()
        acc["eta"] += eta
        acc["retries"] += retries
        ps, pm = ctx.lp_stats()
        acc["piv"] += ps; acc["pmax"] = max(acc["pmax"], pm)
        px = per_x[cur["xi"]]
        px["piv"] += ps; px["n"] += n_local; px["lp"] += tm[0]; px["eta"] += eta
        if not args.no_dedup:
            px["reps"] += ctx.last_push_reps(); px["full"] += ctx.last_push_mode()
        cur["piv"] += ps; cur["lp"] += tm[0]
    t0 = time.perf_counter()
    step_log = []    # per timed step: x index, wall ms, refresh ms, LP kernel ms, mean pivots
    for i in range(args.steps):
        cur["xi"] = i % X
        cur["piv"] = 0; cur["lp"] = 0.0
        ts = time.perf_counter()
        r0 = per_x[i % X]["refresh"]
        alpha = step(xs[i % X], record)
        px = per_x[i % X]
        px["wall"] += time.perf_counter() - ts; px["steps"] += 1; px["alpha"] = alpha
        px["objective"] = step_obj["value"]
        step_log.append([i % X, round(1e3 * (time.perf_counter() - ts), 2), round(1e3 * (px["refresh"] - r0), 2),
                         round(cur["lp"] / 1e3, 2), round(cur["piv"] / max(n_local * E, 1), 3)])
    barrier()
    elapsed = time.perf_counter() - t0
    t_lp, t_dd, t_cut, t_fin, t_sel = acc["lp"], acc["dd"], acc["cut"], acc["fin"], acc["sel"]
    flops_lp, piv_sum, piv_max = acc["flops"], acc["piv"], acc["pmax"]
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=device)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        elapsed = float(t.item())
    K = args.steps
    ms_step = 1e3 * elapsed / K
    value = N * K / elapsed

    # trajectory: K distinct consecutive SD candidates (no revisits), each step refreshing at its
    # new x like a real SD run; timed like the cycle (barrier + synchronize, max over ranks)
    traj = None
    if xs_traj:
        tr_log = []
        tr_piv = 0
        barrier()
        t0 = time.perf_counter()
        for it, xx in zip(traj_iters, xs_traj):
            cur["piv"] = 0; cur["lp"] = 0.0
            ts = time.perf_counter()
            step(xx, lambda: cur.update(piv=cur["piv"] + ctx.lp_stats()[0], lp=cur["lp"] + ctx.timings_us()[0]),
                 per_x_stats=False)
            tr_piv += cur["piv"]
            tr_log.append([it, round(1e3 * (time.perf_counter() - ts), 2), round(cur["lp"] / 1e3, 2),
                           round(cur["piv"] / max(n_local * E, 1), 3), step_obj["value"]])
        barrier()
        el = time.perf_counter() - t0
        if world > 1:
            t = torch.tensor([el], dtype=torch.float64, device=device)
            torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
            el = float(t.item())
        Kt = len(xs_traj)
        traj = {"value": N * Kt / el, "unit": "subproblems/s", "steps": Kt, "ms_per_step": 1e3 * el / Kt,
                "sd_iterations": [traj_iters[0], traj_iters[-1]],
                "rel_step_mean": float(np.mean([np.linalg.norm(b - a) / np.linalg.norm(a)
                                                for a, b in zip([xs[-1]] + xs_traj[:-1], xs_traj)])),
                "lp_pivots_mean": tr_piv / (Kt * max(n_local * E, 1)),
                "steps_log": {"columns": ["sd_iteration", "ms", "lp_kernel_ms", "lp_pivots_mean", "incumbent_objective"],
                              "rows": tr_log},
                "note": "distinct consecutive SD candidates after the cycle's last point, pool refreshed at every x"}

    k = len(positions)
    passes = K * E                 # LP launches / cut passes in the timed region
    # LP kernel (dominant): counted fp64 FLOPs of the executed pivot path per launch
    lp_us = t_lp / passes
    lp_tflops = (flops_lp / passes) / (lp_us * 1e-6) / 1e12
    # cut-gen (argmax + partial sums): algorithmic bytes / flops per pass
    bytes_alg = 8 * n_local * k + 8 * n_local + 12 * n_local + 8 * nv * (m + 1)
    flops_alg = 2 * n_local * nv * k + 2 * nv * m
    cut_us = t_cut / passes
    cut_gbs = bytes_alg / (cut_us * 1e-6) / 1e9
    # the cut's MFMA pass (fp32 by default; fp64 with TWOSD_CUT_F32=0 or out-of-envelope operands)
    cut_fp32, cut_band = ctx.cut_pass()
    peak_cut = PEAK_F32_MFMA_TFS if cut_fp32 else PEAK_FP64_TFS
    t_roof = max(bytes_alg / (PEAK_HBM_GBS * 1e9), flops_alg / (peak_cut * 1e12))
    xnorm = float(np.linalg.norm(xs[0]))
    x_points = [{"x": ("EV (pool training point)" if it == 0 else f"SD candidate, iteration {it}"),
                 "rel_dist_from_ev": float(np.linalg.norm(xx - xs[0]) / xnorm),
                 "steps": px["steps"],
                 "ms_per_step": 1e3 * px["wall"] / max(px["steps"], 1),
                 "pool_refresh_ms": 1e3 * px["refresh"] / max(px["steps"], 1),
                 "pool_refresh_parts_ms": px.get("refresh_parts"),
                 "lp_kernel_ms": px["lp"] / 1e3 / max(px["steps"], 1),
                 "lp_pivots_mean": px["piv"] / max(px["n"], 1),
                 "lp_eta_entries": px["eta"] / max(px["steps"], 1),
                 # the keyed push: duals recovered per epigraph pass, and the passes that recovered
                 # every dual in the main solve instead of re-solving the representatives
                 "push_representatives": px["reps"] / max(px["steps"] * E, 1),
                 "push_full_passes": px["full"],
                 "alpha": px["alpha"],
                 "incumbent_objective": px.get("objective")}
                for it, xx, px in zip(x_iters, xs, per_x)]

    out = {
        "metric": "stage-2 subproblems/sec + cut-gen HBM GB/s on STORM",
        "value": value,
        "unit": "subproblems/s",
        "n_gpus": world,
        "steps": K,
        "warmup": args.warmup,
        "ms_per_step": ms_step,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f64",
        "data": (f"synthetic: i.i.d. scenarios of {name}.sto drawn on the device (Philox4x32-10, seed {args.seed}, "
                 f"{t_gen:.2f} s for the shard)" if args.sampler == "device" else
                 f"synthetic: i.i.d. scenarios of {name}.sto (numpy PCG64, seed {args.seed})") +
                f"; steps cycle over {X} first-stage points (EV + SD candidates, {t_traj:.1f} s to generate)",
        "config": {"workload": f"{name} {N} scenarios" + (f" in {E} epigraphs" if E > 1 else "") +
                               (f" (importance-sampled, scale {args.importance_scale})" if args.importance_scale > 0 else "") +
                               f" sharded over {world} GPU(s), fixed |V|={nv}, " +
                               (f"warm-start pool rebuilt at every new x ({args.refresh_pool} bases from "
                                f"{args.refresh_train} training scenarios, timed), " if args.refresh else
                                f"warm-start pool {pool_size} (trained at x_EV), ") + f"{X} x points, "
                               "LP solve + dual dedup + build_sasa_cut per step",
                   "instance": name, "scenarios": N, "epigraphs": E, "vertices": nv, "k": k, "m2": m,
                   "basis_pool": pool_size, "pool_build_s": round(t_pool, 3),
                   "primary_basis_pivots_mean": round(piv_primary, 2),
                   "pool_refresh": ({"train": args.refresh_train, "pool": args.refresh_pool,
                                     "distributed": dist_refresh} if args.refresh else None),
                   "pool_selection": (f"two-level: {args.pool_level1} + {args.pool_cands} candidates"
                                      if args.pool_level1 > 0 and pool_size > args.pool_level1 else "flat"),
                   "x_points": X,
                   "parallelism": f"scenario-dp{world}"},
        "phases_ms_per_step": {"pool_select": t_sel / K / 1e3, "lp_kernel": t_lp / K / 1e3, "dedup": t_dd / K / 1e3,
                               "cut_partial": t_cut / K / 1e3, "cut_finalize": t_fin / K / 1e3},
        "lp_pivots_mean": piv_sum / (passes * n_local), "lp_pivots_max": piv_max,
        # scenarios of the timed steps whose pool start hit the iteration cap (or numerics) and were
        # solved again from the primary basis
        "lp_iter_limit_retries": acc["retries"],
        "x_points": x_points,
        "steps_log": {"columns": ["x_index", "ms", "refresh_ms", "lp_kernel_ms", "lp_pivots_mean"], "rows": step_log},
        "tie_rule": ("strict '>' (the reference's argmax_procedure, subprob.jl:156)" if args.tie_rel == 0 else
                     f"near-tie: lowest vertex index within {args.tie_rel:g} (1 + |max|) of the maximum"),
        "trajectory": traj,
        "roofline": {"kernel": "lp_hyper_kernel", "bound": "mfma",
                     "note": "fp64 peak (vector == matrix on gfx950); achieved = counted fp64 FLOPs of the executed pivot path / LP kernel time",
                     "achieved": lp_tflops, "peak": PEAK_FP64_TFS, "unit": "TFLOP/s",
                     "frac": lp_tflops / PEAK_FP64_TFS, "traffic": None,
                     # the main launch's eta-arena stores (row index + value per entry): the algorithmic
                     # part of its HBM writes, next to the PMC WRITE_SIZE of the same launch
                     "eta_write_bytes_per_launch": 12.0 * acc["eta"] / passes},
        "cutgen": {"kernel": ("cut_argmax3_kernel (fp32 MFMA pass)" if cut_fp32 else "cut_argmax2_kernel (fp64 MFMA pass)") +
                             " + vbase/pktc/fixup/merge/reduce",
                   "mfma_pass": "fp32" if cut_fp32 else "fp64", "decision_band": cut_band,
                   "peak_tflops": peak_cut, "hbm_gbs": cut_gbs,
                   "bytes_alg": bytes_alg, "flops_alg": flops_alg, "t_roof_ms": t_roof * 1e3,
                   "t_ms": cut_us / 1e3, "frac": t_roof / (cut_us * 1e-6),
                   "mfma_tflops": flops_alg / (cut_us * 1e-6) / 1e12,
                   "bound": "mfma" if flops_alg / (peak_cut * 1e12) > bytes_alg / (PEAK_HBM_GBS * 1e9) else "hbm"},
    }

    # HBM traffic and MFMA counters of the dominant kernels from the committed rocprofv3 PMC
    # summary of this exact workload (separate --pmc passes, tools/profile_round.sh), per launch
    pmc = latest_pmc_summary(name, N, nv, E, world)
    if pmc:
        kl = pmc["kernels"].get("lp_hyper_kernel")
        if kl:
            out["roofline"]["traffic"] = kl["hbm_bytes_per_launch"]
            out["roofline"]["traffic_source"] = pmc["file"]
        kc = pmc["kernels"].get("cut_argmax3_kernel" if cut_fp32 else "cut_argmax2_kernel")
        if kc:
            out["cutgen"]["traffic"] = kc["hbm_bytes_per_launch"]
            if "hbm_bytes_per_launch_raw" in kc:
                out["cutgen"]["traffic_raw"] = kc["hbm_bytes_per_launch_raw"]
            if "mfma_util" in kc:
                out["cutgen"]["mfma_util"] = kc["mfma_util"]            # counted MFMA flops / time / the pass's peak
                out["cutgen"]["mfma_busy_frac"] = kc.get("mfma_busy_frac")   # SQ_VALU_MFMA_BUSY_CYCLES / SIMD cycles
            out["cutgen"]["traffic_source"] = pmc["file"]
    if rank == 0 and world == 1 and args.spot > 0:
        out["parity_spot_check"] = spot_check(sp2, ctx, epi, V, xs, x_iters, positions, args)
    if rank == 0 and world == 1 and args.spot > 0 and not args.no_dedup:
        j = min(1, X - 1)
        out["push_check"] = push_check(ctx, epi, V, nv, xs[j], x_iters[j], n_local, refresh)
    if rank == 0 and world == 1 and not args.no_cpu:
        vals = twosd.get_scenarios(epi, 0, min(n_local, 1 << 19))   # the CPU sample: same scenarios
        out["cpu_baseline"] = cpu_baseline(sp2, ctx, xs, x_iters, heads_at, vals, V.matrix(), args)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


def sd_points(cor, tim, sp2, sto, positions, x_ev, iters, seed, device):
    """First-stage points: x_EV for 0, else the candidate of SD iteration i (sd_iteration!,
    algorithm.jl:39-115: master QP on the host, hot path on this GPU, one scenario per
    iteration from the i.i.d. stream of `seed`), on a context of its own."""
    from sqlp_amd import master, smps, twosd
    out = {0: np.array(x_ev, dtype=np.float64)}
    last = max(iters)
    if last > 0:
        sp1 = smps.get_smps_stage_template(cor, tim, 1)
        c2 = twosd.SDContext(sp2, sto, device=device.index)
        c2.compute_basis(x_ev, smps.mean_values(sto, positions))
        cell = master.sdCell(sp1, c2)
        cell.bind_epigraph(twosd.sdEpigraph(c2, 1.0, 0.0))
        cell.x_candidate = np.array(x_ev, dtype=np.float64)
        cell.x_incumbent = cell.x_candidate.copy()
        rng = np.random.default_rng(seed)
        for it in range(1, last + 1):
            master.sd_iteration(cell, [smps.sample_values(sto, 1, rng, positions)[0]])
            if it in iters:
                out[it] = cell.x_candidate.copy()
        c2.close()
    return [out[i] for i in iters]


def push_check(ctx, epi, V, nv, xx, it, n, refresh):
    """The keyed push of the timed steps vs pushing every scenario's pi (TWOSD_PUSH_ALL=1,
    push! of dual_set.jl:84-94 for s = 1..N in order), over the whole shard at one x point with
    the pool refreshed there: vertex count and the order-dependent fingerprint of V."""
    from sqlp_amd import twosd
    refresh(xx)
    res = {"x_iteration": it, "scenarios": n}
    for key, env in (("keyed", None), ("push_all", "1")):
        V.truncate(nv)
        if env:
            os.environ["TWOSD_PUSH_ALL"] = env
        try:
            twosd.solve_push(epi, xx, 0, n, want_obj=False)
        finally:
            os.environ.pop("TWOSD_PUSH_ALL", None)
        res[key] = {"new_vertices": len(V) - nv, "fingerprint": f"{V.fingerprint():016x}",
                    "pushed": ctx.last_push_reps()}
    V.truncate(nv)
    res["identical"] = (res["keyed"]["new_vertices"] == res["push_all"]["new_vertices"] and
                        res["keyed"]["fingerprint"] == res["push_all"]["fingerprint"])
    return res


def spot_check(sp2, ctx, epi, V, xs, x_iters, positions, args):
    """Parity at bench scale (outside the timed region): the first `spot` scenarios of the
    shard at every x point -- GPU LP objectives vs the C dual simplex (unique optimum), and the
    GPU cut over those scenarios vs the reference-order C argmax/cut with the bench's V."""
    from oracle import cpu
    from sqlp_amd import twosd
    n = min(args.spot, epi.num_scenarios)
    vals = twosd.get_scenarios(epi, 0, n)
    W, T = sp2.dense_W(), sp2.dense_T()
    lp = cpu.CpuLP(W, sp2.q, sp2.sense)
    lp.set_basis(ctx.get_basis())
    rows = ctx.rows
    DR = vals - sp2.r[rows]
    sub = twosd.sdEpigraph(ctx, 1.0, 0.0)
    twosd.add_scenarios(sub, vals)
    Vm = V.matrix()
    threads = max(1, min(16, len(os.sched_getaffinity(0))))
    res = []
    for it, xx in zip(x_iters, xs):
        obj, _, _, st = twosd.solve_batch(sub, xx, 0, n, want_pi=False)
        o_obj, _, _, o_st, _ = lp.solve_batch(rows, sp2.r - T @ xx, DR, nthreads=threads)
        ok = (st == 0) & (o_st == 0)
        lp_err = float(np.max(np.abs(obj[ok] - o_obj[ok]) / (1.0 + np.abs(o_obj[ok])))) if ok.any() else None
        cut = twosd.build_sasa_cut(sub, xx, V, args.tie_rel)
        redecided, cands, full, twins = ctx.cut_stats()
        a, b, omv, _ = cpu.build_cut(sp2.r, T, xx, Vm, rows, DR, np.ones(n), tie_rel=args.tie_rel, nthreads=threads)
        # near ties: scenarios whose two best vertex scores agree to 1e-9 relative (there the strict
        # '>' of the reference picks by the last bits of the summation order, so alpha and beta may
        # differ while the cut value alpha + beta'x = sum_s p_s max_val_s does not)
        scores = (Vm @ (sp2.r - T @ xx))[None, :] + DR @ Vm[:, rows].T
        top2 = np.sort(scores, axis=1)[:, -2:] if Vm.shape[0] > 1 else np.hstack([scores, scores - 1.0])
        ties = int(((top2[:, 1] - top2[:, 0]) <= 1e-9 * (1.0 + np.abs(top2[:, 1]))).sum())
        cv_gpu = cut.alpha + float(cut.beta @ xx)
        cv_cpu = float(np.mean(omv))
        res.append({"x_iteration": it, "scenarios": n, "lp_not_optimal": int((~ok).sum()),
                    "lp_obj_max_rel_err": lp_err,
                    "incumbent_objective_rel_err": abs(float(np.mean(obj[ok])) - float(np.mean(o_obj[ok]))) /
                    (1.0 + abs(float(np.mean(o_obj[ok])))) if ok.any() else None,
                    "cut_value_rel_err": abs(cv_gpu - cv_cpu) / (1.0 + abs(cv_cpu)),
                    "near_tie_scenarios": ties,
                    "cut_redecided": {"scenarios": redecided, "candidates": cands, "full_rescans": full,
                                      "twins_left_out": twins},
                    "alpha_rel_err": abs(cut.alpha - a) / (1.0 + abs(a)),
                    "beta_max_rel_err": float(np.max(np.abs(cut.beta - b)) / (1.0 + np.max(np.abs(b))))})
    return res


def pmc_key(d):
    """The workload a PMC summary was measured on: its "key" (instance, scenarios, vertices,
    epigraphs, n_gpus), or for a summary written before keys existed (profiles/r05) the storm
    bench default it was taken from (|V| = 4096, one epigraph, one GPU)."""
    k = d.get("key")
    if k:
        return (k["instance"], int(k["scenarios"]), int(k["vertices"]), int(k["epigraphs"]), int(k["n_gpus"]))
    return (d.get("workload", "").split(" ")[0], int(d.get("scenarios", 0)), 4096, 1, 1)


def latest_pmc_summary(instance, scenarios, vertices, epigraphs, n_gpus):
    """The newest committed PMC summary (profiles/r*/pmc_summary*.json) of exactly this workload
    -- instance, scenario count, |V|, epigraphs and GPU count -- or None: a line whose workload
    has no profile of its own reports traffic null instead of another workload's counters."""
    import glob
    want = (instance, int(scenarios), int(vertices), int(epigraphs), int(n_gpus))
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", "pmc_summary*.json")))
    for fn in reversed(files):
        with open(fn) as f:
            d = json.load(f)
        if pmc_key(d) == want:
            d["file"] = os.path.relpath(fn, ROOT)
            return d
    return None


def cpu_baseline(sp2, ctx, xs, x_iters, heads_at, vals, Vmat, args):
    """Oracle C restatement on a bounded sample of the same workload (same scenarios, the same
    x points, equal shares of the time budget): warm-started dual simplex + the reference-order
    argmax/cut loops, OpenMP over the host cores.  Two warm starts: (i) the primary basis for
    every scenario, (ii) per scenario the least-infeasible of the first `cpu_pool` bases of the
    GPU's pool at that x (dense inverses built untimed, like the GPU pool's setup).  value = the
    faster of the two."""
    from oracle import cpu
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or len(os.sched_getaffinity(0))
    threads = max(1, min(threads, len(os.sched_getaffinity(0))))
    W = sp2.dense_W()
    T = sp2.dense_T()
    lp = cpu.CpuLP(W, sp2.q, sp2.sense)
    lp.set_basis(ctx.get_basis())
    rows = ctx.rows
    DR = vals - sp2.r[rows]
    chunk = 256 * threads
    budget = args.cpu_seconds / len(xs)
    tot = {"primary_basis": [0, 0.0, 0], "pooled": [0, 0.0, 0]}   # scenarios, seconds, pivots
    at = 0                                                          # next unused sample row

    def timed(solve, key):
        nonlocal at
        n, t, piv = 0, 0.0, 0
        while t < budget and at + chunk <= DR.shape[0]:
            t0 = time.perf_counter()
            it = solve(DR[at:at + chunk])
            t += time.perf_counter() - t0
            piv += int(it.sum())
            n += chunk
            at += chunk
        tot[key][0] += n; tot[key][1] += t; tot[key][2] += piv
        return at - n, n

    t_cut = n_cut = 0
    t_setup = 0.0
    P = 0
    for xi, xx in enumerate(xs):
        base = sp2.r - T @ xx
        a0, n1 = timed(lambda d: lp.solve_batch(rows, base, d, nthreads=threads)[4], "primary_basis")
        t0 = time.perf_counter()
        cpu.build_cut(sp2.r, T, xx, Vmat, rows, DR[a0:a0 + n1], np.ones(n1), tie_rel=args.tie_rel, nthreads=threads)
        t_cut += time.perf_counter() - t0
        n_cut += n1
        heads = heads_at.get(xi)
        if heads is not None and args.cpu_pool > 1 and heads.shape[0] > 1:
            P = heads.shape[0]
            t0 = time.perf_counter()
            lp.set_pool(heads)
            t_setup += time.perf_counter() - t0
            timed(lambda d: lp.solve_batch_pool(rows, base, d, nthreads=threads)[3], "pooled")
    cut_per = t_cut / max(n_cut, 1)
    out = {"unit": "subproblems/s", "cores": threads, "node_cpus": os.cpu_count(), "kind": "port"}
    for key, (n, t, piv) in tot.items():
        if n:
            out[key] = {"value": n / (t + cut_per * n), "scenarios": n, "lp_s": round(t, 3), "lp_pivots_mean": piv / n}
    if "pooled" in out:
        out["pooled"].update({"bases": P, "setup_s": round(t_setup, 2)})
    best = max((k for k in tot if k in out), key=lambda k: out[k]["value"])
    out["value"] = out[best]["value"]
    out["sample"] = (f"{tot['primary_basis'][0]} + {tot['pooled'][0]} storm scenarios of the same stream over the "
                     f"{len(xs)} x points (iterations {x_iters}): C dual simplex from the primary basis "
                     f"({out['primary_basis']['lp_pivots_mean']:.1f} pivots)" +
                     (f" and from the least-infeasible of the GPU pool's first {P} bases at each x "
                      f"({out['pooled']['lp_pivots_mean']:.1f} pivots)" if "pooled" in out else "") +
                     f" + reference-order argmax/cut with |V|={Vmat.shape[0]} ({cut_per * 1e6:.0f} us per scenario); "
                     f"value = {best}")
    return out


if __name__ == "__main__":
    main()

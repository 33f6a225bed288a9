#!/usr/bin/env python3
"""bench.py -- TwoSD scenario-subproblem + cut-generation hot path on MI355X.

Metric (BASELINE.json): stage-2 subproblems/sec + cut-gen HBM GB/s on STORM.
One step = one pass of the hot path over the (sharded) scenario batch at the EV
first-stage x:
  1. solve_problem! for every scenario of the shard (GPU dual simplex, LP kernel),
  2. push! of every dual into the dual vertex set (device dedup), then rollback of the
     set to the fixed |V| pool so every step sees the same set,
  3. build_sasa_cut over the same scenarios with the |V| pool (MFMA argmax + cut),
     RCCL all-reduce of the cut partials when N > 1.
value = scenarios processed by all ranks / max-over-ranks step time.

Workload: storm (data/smps/storm, reference spInput), 1,000,000 i.i.d. synthetic scenarios
from storm.sto (numpy PCG64, per-chunk seeds so any sharding sees the same scenarios),
x = EV solution (tests/golden/ev_x.json), |V| = 4096 real LP duals.  Strong scaling:
the 1M scenarios are split over the ranks.

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
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--instance", default="storm")
    ap.add_argument("--scenarios", type=int, default=1_000_000)
    ap.add_argument("--vertices", type=int, default=4096)
    ap.add_argument("--tie-rel", type=float, default=1e-12)
    ap.add_argument("--seed", type=int, default=20250219)
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="wall budget of the CPU baseline sample")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-dedup", action="store_true")
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
    if args.pool <= 0:
        args.pool = 32768 if args.scenarios // max(1, args.epigraphs) // world >= 500_000 else 16384
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
    while len(V) < args.vertices and at < (1 << 18):
        _, _, pis, st = twosd.solve_batch(src, x, at, 16384, want_pi=True)
        V.push_batch(pis[st == 0])
        at += 16384
    if len(V) > args.vertices:
        V.truncate(args.vertices)
    nv = len(V)

    def step(rec=None):
        ctx.invalidate_x()     # every pass pays its per-x setup (x_B of the pool, selection data)
        alpha = 0.0
        for epi_e, tw in zip(epis, total_weights):
            if args.no_dedup:
                twosd.solve_batch(epi_e, x, 0, n_local, want_pi=False)
            else:
                twosd.solve_push(epi_e, x, 0, n_local)
                V.truncate(nv)
            if world == 1:
                alpha += twosd.build_sasa_cut(epi_e, x, V, args.tie_rel).alpha / E
            else:
                alpha += sdist.build_cut_sharded(ctx, epi_e, x, tw, args.tie_rel, device)[0] / E
            if rec:
                rec()      # per-epigraph kernel timings (HIP events of the last calls)
        return alpha

    def barrier():
        torch.cuda.synchronize(device)
        if world > 1:
            torch.distributed.barrier()
        torch.cuda.synchronize(device)

    for _ in range(args.warmup):
        step()
    barrier()
    acc = {"lp": 0.0, "dd": 0.0, "cut": 0.0, "fin": 0.0, "sel": 0.0, "flops": 0.0, "piv": 0, "pmax": 0}

    def record():
        tm = ctx.timings_us()
        acc["lp"] += tm[0]; acc["dd"] += tm[1]; acc["cut"] += tm[2]; acc["fin"] += tm[3]; acc["sel"] += tm[4]
        acc["flops"] += ctx.lp_flops()
        ps, pm = ctx.lp_stats()
        acc["piv"] += ps; acc["pmax"] = max(acc["pmax"], pm)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        alpha = step(record)
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

    k = len(positions)
    m = sp2.shape[0]
    passes = K * E                 # LP launches / cut passes in the timed region
    # LP kernel (dominant): counted fp64 FLOPs of the executed pivot path per launch
    lp_us = t_lp / passes
    lp_tflops = (flops_lp / passes) / (lp_us * 1e-6) / 1e12
    # cut-gen (argmax + partial sums): algorithmic bytes / flops per pass
    bytes_alg = 8 * n_local * k + 8 * n_local + 12 * n_local + 8 * nv * (m + 1)
    flops_alg = 2 * n_local * nv * k + 2 * nv * m
    cut_us = t_cut / passes
    cut_gbs = bytes_alg / (cut_us * 1e-6) / 1e9
    t_roof = max(bytes_alg / (PEAK_HBM_GBS * 1e9), flops_alg / (PEAK_FP64_TFS * 1e12))

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
                 f"synthetic: i.i.d. scenarios of {name}.sto (numpy PCG64, seed {args.seed})") + ", x = EV solution",
        "config": {"workload": f"{name} {N} scenarios" + (f" in {E} epigraphs" if E > 1 else "") +
                               (f" (importance-sampled, scale {args.importance_scale})" if args.importance_scale > 0 else "") +
                               f" sharded over {world} GPU(s), |V|={nv}, "
                               f"warm-start pool {pool_size}, LP solve + dual dedup + build_sasa_cut per step",
                   "instance": name, "scenarios": N, "epigraphs": E, "vertices": nv, "k": k, "m2": m,
                   "basis_pool": pool_size, "pool_build_s": round(t_pool, 3),
                   "pool_selection": (f"two-level: {args.pool_level1} + {args.pool_cands} candidates"
                                      if args.pool_level1 > 0 and pool_size > args.pool_level1 else "flat"),
                   "parallelism": f"scenario-dp{world}"},
        "phases_ms_per_step": {"pool_select": t_sel / K / 1e3, "lp_kernel": t_lp / K / 1e3, "dedup": t_dd / K / 1e3,
                               "cut_partial": t_cut / K / 1e3, "cut_finalize": t_fin / K / 1e3},
        "lp_pivots_mean": piv_sum / (passes * n_local), "lp_pivots_max": piv_max,
        "roofline": {"kernel": "lp_hyper_kernel", "bound": "mfma",
                     "note": "fp64 peak (vector == matrix on gfx950); achieved = counted fp64 FLOPs of the executed pivot path / LP kernel time",
                     "achieved": lp_tflops, "peak": PEAK_FP64_TFS, "unit": "TFLOP/s",
                     "frac": lp_tflops / PEAK_FP64_TFS, "traffic": None},
        "cutgen": {"kernel": "cut_argmax_kernel (+vbase/fixup/reduce)", "hbm_gbs": cut_gbs,
                   "bytes_alg": bytes_alg, "flops_alg": flops_alg, "t_roof_ms": t_roof * 1e3,
                   "t_ms": cut_us / 1e3, "frac": t_roof / (cut_us * 1e-6),
                   "bound": "mfma" if flops_alg / (PEAK_FP64_TFS * 1e12) > bytes_alg / (PEAK_HBM_GBS * 1e9) else "hbm"},
        "alpha_check": alpha,
    }

    # measured peaks of this part (tools/mfma_f64_probe.hip, committed under profiles/): the
    # fp64 MFMA and VALU rates reach ~60 % / ~88 % of the spec, so both fractions are reported
    peaks = latest_peaks()
    if peaks:
        vf = max((p["tflops"] for p in peaks if p["probe"] == "v_fma_f64"), default=None)
        mf = max((p["tflops"] for p in peaks if p["probe"].startswith("mfma_f64")), default=None)
        if vf:
            out["roofline"].update({"peak_measured": vf, "frac_measured": lp_tflops / vf,
                                    "peak_measured_source": "v_fma_f64 probe, " + peaks[0]["file"]})
        if mf:
            out["cutgen"].update({"mfma_tflops": flops_alg / (cut_us * 1e-6) / 1e12, "peak_measured_tflops": mf,
                                  "frac_measured": flops_alg / (cut_us * 1e-6) / 1e12 / mf,
                                  "peak_measured_source": "mfma_f64_16x16x4f64 probe, " + peaks[0]["file"]})

    # HBM traffic of the dominant kernel from the committed rocprofv3 PMC summary of this exact
    # workload (separate --pmc passes, tools/profile_round.sh), per launch like `achieved`
    pmc = latest_pmc_summary()
    if pmc and world == 1 and pmc.get("scenarios") == N:
        k = pmc["kernels"].get("lp_hyper_kernel")
        if k:
            out["roofline"]["traffic"] = k["hbm_bytes_per_launch"]
            out["roofline"]["traffic_source"] = pmc["file"]
        kc = pmc["kernels"].get("cut_argmax_kernel")
        if kc:
            out["cutgen"]["traffic"] = kc["hbm_bytes_per_launch"]
    if rank == 0 and world == 1 and not args.no_cpu:
        vals = twosd.get_scenarios(epi, 0, min(n_local, 1 << 19))   # the CPU sample: same scenarios
        out["cpu_baseline"] = cpu_baseline(sp2, ctx, x, vals, V.matrix(), positions, args)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


def latest_peaks():
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", "peaks.jsonl")))
    if not files:
        return None
    with open(files[-1]) as f:
        rows = [json.loads(l) for l in f if l.strip()]
    for r in rows:
        r["file"] = os.path.relpath(files[-1], ROOT)
    return rows


def latest_pmc_summary():
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", "pmc_summary.json")))
    if not files:
        return None
    with open(files[-1]) as f:
        d = json.load(f)
    d["file"] = os.path.relpath(files[-1], ROOT)
    d.setdefault("scenarios", 1_000_000)
    return d


def cpu_baseline(sp2, ctx, x, vals, Vmat, positions, args):
    """Oracle C restatement (warm-started dual simplex from the same basis + the
    reference-order argmax/cut loops) on a bounded sample of the same workload."""
    from oracle import cpu
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or len(os.sched_getaffinity(0))
    threads = max(1, min(threads, len(os.sched_getaffinity(0))))
    W = sp2.dense_W()
    T = sp2.dense_T()
    lp = cpu.CpuLP(W, sp2.q, sp2.sense)
    lp.set_basis(ctx.get_basis())
    rows = ctx.rows
    base = sp2.r - T @ x
    DR = vals - sp2.r[rows]
    n_done, t_lp = 0, 0.0
    chunk = 256 * threads
    while t_lp < args.cpu_seconds and n_done + chunk <= DR.shape[0]:
        t0 = time.perf_counter()
        lp.solve_batch(rows, base, DR[n_done:n_done + chunk], nthreads=threads)
        t_lp += time.perf_counter() - t0
        n_done += chunk
    t0 = time.perf_counter()
    cpu.build_cut(sp2.r, T, x, Vmat, rows, DR[:n_done], np.ones(n_done), tie_rel=args.tie_rel, nthreads=threads)
    t_cut = time.perf_counter() - t0
    return {"value": n_done / (t_lp + t_cut), "unit": "subproblems/s", "cores": threads, "kind": "port",
            "sample": f"{n_done} storm scenarios of the same stream: warm-started C dual simplex "
                      f"({t_lp:.2f}s) + reference-order argmax/cut with |V|={Vmat.shape[0]} ({t_cut:.2f}s)"}


if __name__ == "__main__":
    main()

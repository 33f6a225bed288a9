"""Diagnostic: phase shares of the LP kernel at the bench configuration (storm, device-drawn
scenarios, two-level basis pool).  Run with TWOSD_LIB=stamps (libtwosd_hip_stamps.so, built
by `make -C sqlp_amd/csrc stamps`); the stamps perturb the schedule, so only the shares and
the cycles per pivot are meaningful, never the absolute kernel time.

usage: TWOSD_LIB=stamps python tools/lp_phases_bench.py [N] [pool] [batch|push]
(push: the keyed solve_push of the bench -- dual keys instead of pi, recovery for the
representatives only; the stamps then cover the main launch and the re-solves)
"""
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from tools.lp_phases import PHASES  # noqa: E402


def main():
    from sqlp_amd import smps, twosd
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 250000
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
    tr = twosd.sdEpigraph(ctx, 1.0, 0.0)
    twosd.add_sampled_scenarios(tr, 4 * pool, seed + 2)
    ctx.pool_build(tr, x, 0, 4 * pool, pool)
    ct = twosd.sdEpigraph(ctx, 1.0, 0.0)
    twosd.add_sampled_scenarios(ct, 262144, seed + 3)
    ctx.pool_build_candidates(ct, x, 0, 262144, 128, 160)
    epi = twosd.sdEpigraph(ctx, 1.0, 0.0)
    twosd.add_sampled_scenarios(epi, N, seed)
    twosd.solve_batch(epi, x, 0, min(N, 4096), want_pi=False)
    st = np.zeros(10, dtype=np.uint64)
    ctx.lib.twosd_debug_stamps(ctx.h, st.ctypes.data_as(C.c_void_p), 1)
    mode = sys.argv[3] if len(sys.argv) > 3 else "batch"
    if mode == "push":
        V = twosd.sdDualVertexSet(ctx)
        twosd.solve_push(epi, x, 0, N, want_obj=False)
        print(f"representatives re-solved: {ctx.last_push_reps()}, |V| = {len(V)}")
    else:
        twosd.solve_batch(epi, x, 0, N, want_pi=True)
    ctx.lib.twosd_debug_stamps(ctx.h, st.ctypes.data_as(C.c_void_p), 1)
    tot = float(st.sum())
    t = ctx.timings_us()
    piv, pmax = ctx.lp_stats()
    print(f"{name} N={N} pool={ctx.pool_size()} lp_kernel_ms={t[0] / 1e3:.2f} pivots/scen={piv / N:.2f} "
          f"cycles/scenario/wave={tot / N:.0f}")
    for p, v in zip(PHASES, st):
        print(f"  {p:18s} {100 * v / tot:6.2f}%  {v / N:10.0f} cyc/scenario")


if __name__ == "__main__":
    main()

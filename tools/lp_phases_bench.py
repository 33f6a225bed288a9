"""Diagnostic: phase shares of the LP kernel at the bench configuration (storm, device-drawn
scenarios, per-x pool refresh of 4096 bases from 16384 training solves, two-level selection,
keyed solve_push), at each of the bench's x points.  Run with TWOSD_LIB=stamps
(libtwosd_hip_stamps.so, built by `make -C sqlp_amd/csrc stamps`); the stamps perturb the
schedule, so only the shares and the cycles per scenario are meaningful, never the absolute
kernel time.

usage: TWOSD_LIB=stamps python tools/lp_phases_bench.py [N] [pool] [train] [instance (storm)]
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
    import torch
    torch.cuda.init()
    import bench
    from sqlp_amd import smps, twosd
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 250000
    P = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
    T = int(sys.argv[3]) if len(sys.argv) > 3 else 4 * P
    inst = sys.argv[4] if len(sys.argv) > 4 else "storm"
    seed = 20250219
    d = os.path.join(ROOT, "data", "smps", inst)
    cor, tim, sto = smps.load_smps(d, inst)
    sp2 = smps.get_smps_stage_template(cor, tim, 2)
    with open(os.path.join(ROOT, "tests", "golden", "ev_x.json")) as f:
        x0 = np.array(json.load(f)[inst]["x"])
    positions = list(sto.indep.keys())
    its = [0, 4, 12, 30]
    xs = bench.sd_points(cor, tim, sp2, sto, positions, x0, its, seed + 7, torch.device("cuda", 0))
    ctx = twosd.SDContext(sp2, sto)
    ctx.compute_basis(x0, smps.mean_values(sto, positions))
    ctx.set_distributions(sto)
    tr = twosd.sdEpigraph(ctx, 1.0, 0.0)
    twosd.add_sampled_scenarios(tr, T, seed + 4)
    epi = twosd.sdEpigraph(ctx, 1.0, 0.0)
    twosd.add_sampled_scenarios(epi, N, seed)
    twosd.sdDualVertexSet(ctx)
    ctx.pool_refresh(tr, xs[-1], 0, T, P)
    st = np.zeros(10, dtype=np.uint64)
    tot_all = np.zeros(10)
    for it, xx in zip(its, xs):
        ctx.pool_refresh(tr, xx, 0, T, P)
        ctx.pool_build_candidates(tr, xx, 0, T, 128, 160)
        ctx.lib.twosd_debug_stamps(ctx.h, st.ctypes.data_as(C.c_void_p), 1)    # reset
        twosd.solve_push(epi, xx, 0, N, want_obj=False)
        piv = ctx.lp_stats()[0] / N       # the main launch (the representatives' re-solve is separate)
        ctx.lib.twosd_debug_stamps(ctx.h, st.ctypes.data_as(C.c_void_p), 1)
        tot = float(st.sum())
        tot_all += st
        print(f"x{it}: pivots/scen {piv:.2f}, representatives {ctx.last_push_reps()}, "
              f"cycles/scenario/wave {tot / N:.0f} | " +
              " ".join(f"{p} {100 * v / tot:.1f}%" for p, v in zip(PHASES, st)), flush=True)
    tot = tot_all.sum()
    print("all x points:")
    for p, v in zip(PHASES, tot_all):
        print(f"  {p:18s} {100 * v / tot:6.2f}%  {v / (len(its) * N):10.0f} cyc/scenario")


if __name__ == "__main__":
    main()

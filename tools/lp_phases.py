"""Diagnostic: where the hypersparse LP kernel spends its cycles (phase-stamp build).

Run with TWOSD_LIB=stamps (libtwosd_hip_stamps.so, built by `make -C sqlp_amd/csrc stamps`).
Prints per-phase shares of the summed wave cycles; the stamp build perturbs the schedule,
so only the shares are meaningful, never the absolute time.
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

PHASES = ["init_xB", "leaving_row", "btran_etas", "rho_scatter", "pricing", "harris_ratio", "dual_update",
          "ftran", "updates", "final_recovery"]


def main():
    import ctypes as C
    from sqlp_amd import smps, twosd
    name = sys.argv[1] if len(sys.argv) > 1 else "storm"
    N = int(sys.argv[2]) if len(sys.argv) > 2 else 20000
    d = os.path.join(ROOT, "data", "smps", name)
    cor, tim, sto = smps.load_smps(d, name)
    sp2 = smps.get_smps_stage_template(cor, tim, 2)
    with open(os.path.join(ROOT, "tests", "golden", "ev_x.json")) as f:
        x = np.array(json.load(f)[name]["x"])
    ctx = twosd.SDContext(sp2, sto)
    ctx.compute_basis(x, smps.mean_values(sto))
    vals = smps.sample_values(sto, N, np.random.default_rng(1))
    pool = int(os.environ.get("POOL", "1"))
    if pool > 1:
        tr = twosd.sdEpigraph(ctx, 1.0, 0.0)
        twosd.add_scenarios(tr, smps.sample_values(sto, 16384, np.random.default_rng(99)))
        ctx.pool_build(tr, x, 0, 16384, pool)
    ctx.solve_values(x, vals[:1024], want_pi=False)
    st = np.zeros(10, dtype=np.uint64)
    ctx.lib.twosd_debug_stamps(ctx.h, st.ctypes.data_as(C.c_void_p), 1)
    ctx.solve_values(x, vals, want_pi=False)
    ctx.lib.twosd_debug_stamps(ctx.h, st.ctypes.data_as(C.c_void_p), 1)
    tot = float(st.sum())
    t = ctx.timings_us()
    piv, pmax = ctx.lp_stats()
    print(f"{name} N={N} lp_kernel_ms={t[0] / 1e3:.2f} pivots/scen={piv / N:.1f} cycles/pivot/wave={tot / max(piv, 1):.0f}")
    for p, v in zip(PHASES, st):
        print(f"  {p:18s} {100 * v / tot:6.2f}%  {v / max(piv, 1):10.0f} cyc/pivot")


if __name__ == "__main__":
    main()

"""Development timing of the LP batch alone: python tools/lp_speed.py <instance> <N> [reps].
Prints LP kernel ms (HIP events), scenarios/s and pivots; honours TWOSD_LIB / TWOSD_LP_KERNEL."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def solve_nocheck(twosd, epi, x, N):
    """solve_batch without raising on non-optimal scenarios (status reported instead)."""
    import ctypes as C
    ctx = epi.ctx
    obj = np.zeros(N)
    st = np.zeros(N, dtype=np.int32)
    xx = np.ascontiguousarray(x, dtype=np.float64)
    p = lambda a: a.ctypes.data_as(C.c_void_p)
    rc = ctx.lib.twosd_solve_batch(ctx.h, epi.index, p(xx), 0, N, p(obj), None, None, p(st))
    if rc not in (0, -4):   # TWOSD_OK, TWOSD_E_LP
        raise RuntimeError(f"twosd_solve_batch rc={rc}")
    return obj, st


def main():
    from sqlp_amd import smps, twosd
    name = sys.argv[1] if len(sys.argv) > 1 else "storm"
    N = int(sys.argv[2]) if len(sys.argv) > 2 else 100000
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    d = os.path.join(ROOT, "data", "smps", name)
    cor, tim, sto = smps.load_smps(d, name)
    sp2 = smps.get_smps_stage_template(cor, tim, 2)
    with open(os.path.join(ROOT, "tests", "golden", "ev_x.json")) as f:
        x = np.array(json.load(f)[name]["x"])
    ctx = twosd.SDContext(sp2, sto)
    ctx.compute_basis(x, smps.mean_values(sto))
    vals = smps.sample_values(sto, N, np.random.default_rng(1))
    pool = int(os.environ.get("POOL", "1"))
    if pool > 1:   # warm-start basis pool from independent training scenarios
        tr = twosd.sdEpigraph(ctx, 1.0, 0.0)
        ntr = int(os.environ.get("POOL_TRAIN", "16384"))
        twosd.add_scenarios(tr, smps.sample_values(sto, ntr, np.random.default_rng(99)))
        import time
        t0 = time.perf_counter()
        ctx.pool_build(tr, x, 0, ntr, pool)
        print(f"pool size {ctx.pool_size()} built in {time.perf_counter() - t0:.2f} s")
    epi = twosd.sdEpigraph(ctx, 1.0, 0.0)
    twosd.add_scenarios(epi, vals)
    solve_nocheck(twosd, epi, x, min(N, 4096))
    ts, walls = [], []
    import time
    for rep in range(reps):
        # XALT=1: alternate x between reps (per-x host preparation inside the wall time)
        xr = x * (1.0 + 1e-3 * (rep % 2)) if os.environ.get("XALT") else x
        t0 = time.perf_counter()
        obj, st = solve_nocheck(twosd, epi, xr, N)
        walls.append((time.perf_counter() - t0) * 1e3)
        tm = ctx.timings_us()
        ts.append((tm[0] + tm[4]) / 1e3)   # pool selection + LP kernel
    piv, pmax = ctx.lp_stats()
    t = min(ts)
    print(f"{os.environ.get('TWOSD_LIB', 'default')} {name} N={N} lp_ms={t:.2f} ({' '.join(f'{v:.1f}' for v in ts)}) "
          f"scen/s={N / t * 1e3:.0f} pivots/scen={piv / N:.2f} max={pmax} status_ok={(st == 0).mean():.6f} bad={np.flatnonzero(st)[:5].tolist()} st={np.unique(st).tolist()} "
          f"objsum={obj.sum():.6e} wall_ms={' '.join(f'{v:.1f}' for v in walls)}")


if __name__ == "__main__":
    main()

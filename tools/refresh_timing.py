"""Diagnostic: phase timings of one pool refresh at an SD candidate point (run with
TWOSD_DEBUG=1 for the upload breakdown).  usage: python tools/refresh_timing.py [T] [max_pool]"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import bench
    from sqlp_amd import smps, twosd
    T = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
    mp = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
    name = "storm"
    d = os.path.join(ROOT, "data", "smps", name)
    cor, tim, sto = smps.load_smps(d, name)
    sp2 = smps.get_smps_stage_template(cor, tim, 2)
    with open(os.path.join(ROOT, "tests", "golden", "ev_x.json")) as f:
        x_ev = np.array(json.load(f)[name]["x"])
    positions = list(sto.indep.keys())
    seed = 20250219
    xs = bench.sd_points(cor, tim, sp2, sto, positions, x_ev, [4, 12], seed + 7, torch.device("cuda", 0))
    ctx = twosd.SDContext(sp2, sto)
    ctx.compute_basis(x_ev, smps.mean_values(sto, positions))
    ctx.set_distributions(sto)
    tr = twosd.sdEpigraph(ctx, 1.0, 0.0)
    twosd.add_sampled_scenarios(tr, 16384, seed + 2)
    ctx.pool_build(tr, x_ev, 0, 16384, 4096)
    rt = twosd.sdEpigraph(ctx, 1.0, 0.0)
    twosd.add_sampled_scenarios(rt, T, seed + 5)
    for xx in xs:
        t0 = time.perf_counter()
        n = ctx.pool_refresh(rt, xx, 0, T, mp)
        print(f"refresh pool={n} wall {1e3 * (time.perf_counter() - t0):.1f} ms, phases {ctx.last_refresh_ms()}", flush=True)


if __name__ == "__main__":
    main()

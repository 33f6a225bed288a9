"""Diagnostic: how many bases of the refreshed pool at each bench x point were already in the pool
it was trained from (same set of basic columns).  usage: python tools/pool_overlap.py"""
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
    prev = None
    for rnd in range(2):
        for xi in (1, 2, 3, 0):
            ctx.pool_refresh(tr, xs[xi], 0, T, P)
            keys = {tuple(sorted(ctx.pool_get(p))) for p in range(ctx.pool_size())}
            if prev is not None:
                print(f"round {rnd} x{xi}: pool {len(keys)}, already in the previous pool {len(keys & prev)}", flush=True)
            prev = keys


if __name__ == "__main__":
    main()

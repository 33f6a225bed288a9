"""Twin-context determinism check (development): two contexts built the same way run the bench's
pool protocol step by step (refresh, candidate build, LP batch at each x); after every step their
pools and LP outputs are compared, so the first step whose result depends on anything but its
inputs (uninitialised device memory, timing) is named.
Usage (GPU box): python -u tools/lp_twin.py [N] [train] [pool] [push]"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import bench
    from sqlp_amd import smps, twosd
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 200000
    TR = int(sys.argv[2]) if len(sys.argv) > 2 else 16384
    POOL = int(sys.argv[3]) if len(sys.argv) > 3 else 4096
    PUSH = len(sys.argv) > 4 and sys.argv[4] == "push"   # the bench's step: keyed push + cut
    name = "storm"
    d = os.path.join(ROOT, "data", "smps", name)
    cor, tim, sto = smps.load_smps(d, name)
    sp2 = smps.get_smps_stage_template(cor, tim, 2)
    with open(os.path.join(ROOT, "tests", "golden", "ev_x.json")) as f:
        x0 = np.array(json.load(f)[name]["x"])
    positions = list(sto.indep.keys())
    xs = bench.sd_points(cor, tim, sp2, sto, positions, x0, [0, 4, 12, 30], 20250219 + 7, torch.device("cuda", 0))
    print("points ready", flush=True)

    def make():
        ctx = twosd.SDContext(sp2, sto)
        ctx.compute_basis(x0, smps.mean_values(sto, positions))
        ctx.set_distributions(sto)
        epi = twosd.sdEpigraph(ctx, 1.0, 0.0)
        twosd.add_sampled_scenarios(epi, N, 20250219)
        tr = twosd.sdEpigraph(ctx, 1.0, 0.0)
        twosd.add_sampled_scenarios(tr, TR, 20250223)
        V = twosd.sdDualVertexSet(ctx)
        src = twosd.sdEpigraph(ctx, 1.0, 0.0)
        twosd.add_sampled_scenarios(src, 1 << 16, 20250220)
        at = 0
        while len(V) < 4096 and at < (1 << 16):
            _, _, pis, st = twosd.solve_batch(src, x0, at, 16384, want_pi=True)
            V.push_batch(pis[st == 0])
            at += 16384
        V.truncate(min(4096, len(V)))
        return ctx, epi, tr, V

    A, B = make(), make()

    def pools(ctx):
        return np.stack([ctx.pool_get(p) for p in range(ctx.pool_size())])

    step = 0
    for rnd in range(2):
        for i, xx in enumerate(xs):
            outs = []
            for ctx, epi, tr, V in (A, B):
                ctx.pool_refresh(tr, xx, 0, TR, POOL)
                p1 = pools(ctx)
                ctx.pool_build_candidates(tr, xx, 0, TR, 128, 160)
                if PUSH:
                    nv = len(V)
                    twosd.solve_push(epi, xx, 0, N, want_obj=False)
                    V.truncate(nv)
                    c = twosd.build_sasa_cut(epi, xx, V, 0.0)
                    obj = np.array([c.alpha]); st = np.zeros(1, np.int32)
                else:
                    obj, _, _, st = twosd.solve_batch(epi, xx, 0, N, want_pi=False)
                it = ctx.last_lp_iters(N)[0].copy()
                pk = ctx.last_pool_picks(N).copy()
                outs.append((p1, obj.view(np.int64).copy(), st.copy(), it, pk))
            a, b = outs
            same_pool = a[0].shape == b[0].shape and bool((a[0] == b[0]).all())
            nd = 0 if not (a[0].shape == b[0].shape) else int((a[0] != b[0]).any(1).sum())
            print(json.dumps({"step": step, "round": rnd, "x": i, "pool_sizes": [a[0].shape[0], b[0].shape[0]],
                              "pools_identical": same_pool, "pool_rows_differ": nd,
                              "picks_differ": int((a[4] != b[4]).sum()), "iters_differ": int((a[3] != b[3]).sum()),
                              "obj_bits_differ": int((a[1] != b[1]).sum()),
                              "mean_iters": [round(float(a[3].mean()), 3), round(float(b[3].mean()), 3)]}), flush=True)
            step += 1


if __name__ == "__main__":
    main()

"""How many vertices fall in the fp32 pass's decision band per scenario (storm at x_EV, |V| = 4096):
the global band (one radius for every vertex: the cut's band) against per-vertex radii
e_v = band/2 * a_v / max a (a_v = sum_e |PK[v,e] coef_e| dmax_e, the quantity the band scales).
Exact fp64 scores of N scenarios in numpy (the candidates' count, not the kernel's arithmetic).
usage: python tools/band_study.py [N]"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    from sqlp_amd import smps, twosd
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 20000
    name = "storm"
    d = os.path.join(ROOT, "data", "smps", name)
    cor, tim, sto = smps.load_smps(d, name)
    sp2 = smps.get_smps_stage_template(cor, tim, 2)
    with open(os.path.join(ROOT, "tests", "golden", "ev_x.json")) as f:
        x = np.array(json.load(f)[name]["x"])
    ctx = twosd.SDContext(sp2, sto)
    ctx.compute_basis(x, smps.mean_values(sto))
    ctx.set_distributions(sto)
    src = twosd.sdEpigraph(ctx, 1.0, 0.0)
    twosd.add_sampled_scenarios(src, 1 << 18, 20250220)
    V = twosd.sdDualVertexSet(ctx)
    at = 0
    while len(V) < 4096 and at < (1 << 18):
        _, _, pis, st = twosd.solve_batch(src, x, at, 16384, want_pi=True)
        V.push_batch(pis[st == 0])
        at += 16384
    V.truncate(min(len(V), 4096))
    big = twosd.sdEpigraph(ctx, 1.0, 0.0)
    twosd.add_sampled_scenarios(big, 1000000, 20250219)
    twosd.build_sasa_cut(big, x, V, 0.0)
    fp32, band = ctx.cut_pass()
    rows = ctx.rows
    vals = twosd.get_scenarios(big, 0, N)
    DR = vals - sp2.r[rows]
    Vm = V.matrix()
    T = sp2.dense_T()
    base = Vm @ (sp2.r - T @ x)
    PK = Vm[:, rows]                     # RHS randomness: coef_e = 1
    dmax = np.abs(twosd.get_scenarios(big, 0, 200000) - sp2.r[rows]).max(axis=0)
    a = np.abs(PK) @ dmax
    S = base[None, :] + DR @ PK.T
    M = S.max(axis=1, keepdims=True)
    n_glob = (S >= M - band).sum(axis=1)
    e = 0.5 * band * a / a.max()
    L = (S - e[None, :]).max(axis=1, keepdims=True)
    n_pv = (S + e[None, :] >= L).sum(axis=1)
    q = np.quantile(a / a.max(), [0.0, 0.1, 0.25, 0.5, 0.75, 0.9, 1.0])
    print(json.dumps({"N": N, "V": len(V), "fp32": fp32, "band": band, "a_over_max_quantiles": [round(float(v), 4) for v in q],
                      "global_band": {"mean_candidates": float(n_glob.mean()), "rows_decided": float((n_glob == 1).mean())},
                      "per_vertex": {"mean_candidates": float(n_pv.mean()), "rows_decided": float((n_pv == 1).mean())},
                      "score_spread_top2_median": float(np.median(np.sort(S, axis=1)[:, -1] - np.sort(S, axis=1)[:, -2]))}))


if __name__ == "__main__":
    main()

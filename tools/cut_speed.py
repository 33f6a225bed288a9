"""Development timing of build_sasa_cut alone (storm, device-drawn scenarios, |V| real duals).
usage: [TWOSD_LIB=variant] [TIE_REL=t] python tools/cut_speed.py [N] [|V|] [reps]"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    from sqlp_amd import smps, twosd
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 1000000
    nvt = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 5
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
    while len(V) < nvt and at < (1 << 18):
        _, _, pis, st = twosd.solve_batch(src, x, at, 16384, want_pi=True)
        V.push_batch(pis[st == 0])
        at += 16384
    V.truncate(min(len(V), nvt))
    epi = twosd.sdEpigraph(ctx, 1.0, 0.0)
    twosd.add_sampled_scenarios(epi, N, 20250219)
    ts = []
    tie = float(os.environ.get("TIE_REL", "0"))
    for _ in range(reps):
        ctx.invalidate_x()
        cut = twosd.build_sasa_cut(epi, x, V, tie)
        ts.append(ctx.timings_us()[2] / 1e3)
    stats = ctx.cut_stats()   # (re-decided scenarios, candidates, full re-scans, twins left out) of the last cut
    k = len(ctx.rows)
    flops = 2 * N * len(V) * k + 2 * len(V) * sp2.shape[0]
    t = min(ts)
    print(json.dumps({"lib": os.environ.get("TWOSD_LIB", "default"), "N": N, "V": len(V), "cut_ms": ts,
                      "tflops": flops / (t * 1e-3) / 1e12, "frac": flops / (t * 1e-3) / 78.6e12, "alpha": cut.alpha,
                      "tie_rel": tie, "redecided": stats}))


if __name__ == "__main__":
    main()

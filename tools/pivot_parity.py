"""Pivot-path agreement of the LP kernel with the C oracle (same rules, same start basis):
storm scenarios from the primary basis at x_EV, per-scenario pivots and vertices compared.
A build whose arithmetic drifts from the oracle's shows it here before it shows in pool
statistics.  Usage (GPU box): [TWOSD_LIB=variant] python tools/pivot_parity.py [N] [instance]"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    from oracle import cpu
    from sqlp_amd import smps, twosd
    from tests import instances as I
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 3000
    name = sys.argv[2] if len(sys.argv) > 2 else "storm"
    inst = I.load(name)
    sp2, sto = inst["sp2"], inst["sto"]
    x = I.x_ev(name)
    ctx = twosd.SDContext(sp2, sto)
    positions = list(sto.indep.keys())
    ctx.compute_basis(x, smps.mean_values(sto, positions))
    vals = I.sample(name, N, seed=7)
    obj, _, pi, st = ctx.solve_values(x, vals, want_pi=True)
    its, _ = ctx.last_lp_iters(N)
    sp = inst["osp2"]
    lp = cpu.CpuLP(sp.W, sp.q, sp.senses)
    lp.set_basis(ctx.get_basis())
    pos, rows, cols = smps.scenario_positions(sp2, sto)
    o_obj, o_pi, _, o_st, o_it = lp.solve_batch(rows, sp.r - sp.T @ x, vals - sp.r[rows], nthreads=8)
    ok = (st == 0) & (o_st == 0)
    same_v = np.all(np.abs(pi - o_pi) <= 1e-9 * (1 + np.abs(o_pi)), axis=1)
    print(f"{name} N={N} lib={os.environ.get('TWOSD_LIB', 'default')}: GPU pivots {its.mean():.3f}, oracle {o_it.mean():.3f}, "
          f"equal pivot counts {np.mean(its == o_it):.4f}, same vertex {np.mean(same_v[ok]):.4f}, "
          f"max obj rel err {np.max(np.abs(obj - o_obj) / (1 + np.abs(o_obj))):.2e}", flush=True)


if __name__ == "__main__":
    main()

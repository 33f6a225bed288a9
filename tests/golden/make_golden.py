"""Generate the golden fixtures under tests/golden/ (run from the repo root:
``python tests/golden/make_golden.py``).

Generator: the oracle restatement (oracle/smps_ref.py, oracle/twosd_ref.py) and HiGHS
(scipy 1.15.3, oracle/lp_highs.py) -- the reference itself (Julia/JuMP/GLPK) cannot run
here.  Every fixture stores explicit scenario values, never RNG seeds (Julia's RNG stream
cannot be matched).  Files:
  ev_x.json          first-stage x of the expected-value problem (+ EV objective) per instance
  lp_<name>.npz      x, scenario values, HiGHS obj / duals for a handful of scenarios
  cut_<name>.npz     V (HiGHS duals), x, values, weights, reference-order build_sasa_cut
                     alpha / beta / max_val / max_arg (strict '>' rule, tie_rel = 0)
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle import lp_highs, smps_ref, twosd_ref  # noqa: E402

DATA = os.path.join(ROOT, "data", "smps")
NAMES = ["lands", "newsvendor", "transship", "ssn", "storm", "baa99-20"]
N_LP = {"lands": 12, "newsvendor": 10, "transship": 16, "ssn": 16, "storm": 12, "baa99-20": 12}
N_CUT = {"lands": 12, "newsvendor": 10, "transship": 24, "ssn": 24, "storm": 16, "baa99-20": 16}


def sample(sto, N, rng):
    out = np.empty((N, len(sto.indep)))
    for e, (pos, d) in enumerate(sto.indep.items()):
        if d[0] == "DISCRETE":
            out[:, e] = rng.choice(np.array(d[1]), size=N, p=np.array(d[2]) / np.sum(d[2]))
        elif d[0] == "NORMAL":
            out[:, e] = rng.normal(d[1], np.sqrt(d[2]), size=N)
        else:
            out[:, e] = rng.uniform(d[1], d[2], size=N)
    return out


def main():
    ev = {}
    for name in NAMES:
        cor, tim, sto = smps_ref.load_instance(os.path.join(DATA, name), name)
        sp1 = smps_ref.stage_template(cor, tim, 1)
        sp2 = smps_ref.stage_template(cor, tim, 2)
        evobj, x = lp_highs.solve_ev(sp1, sp2, lp_highs.sto_mean_rhs(sp2, sto))
        ev[name] = {"x": [float(t) for t in x], "ev_obj": evobj}
        rowm = {n: i for i, n in enumerate(sp2.row_names)}
        rows = np.array([rowm[p[1]] for p in sto.indep], dtype=np.int64)
        rng = np.random.default_rng(20250219 + len(name))
        vals = sample(sto, N_LP[name], rng)
        objs, pis = [], []
        for v in vals:
            r = sp2.r.copy(); r[rows] = v
            st, o, y, pi = lp_highs.solve_problem(sp2, x, r)
            assert st == 0, (name, st)
            objs.append(o); pis.append(pi)
        np.savez_compressed(os.path.join(HERE, f"lp_{name}.npz"), x=x, values=vals, rows=rows,
                            obj=np.array(objs), pi=np.array(pis))
        # cut fixture: V from HiGHS duals of other scenarios, reference-order cut
        vals_c = sample(sto, N_CUT[name], rng)
        Vset = twosd_ref.DualVertexSet()
        for v in sample(sto, 2 * N_CUT[name], rng):
            r = sp2.r.copy(); r[rows] = v
            st, o, y, pi = lp_highs.solve_problem(sp2, x, r)
            Vset.push(pi)
        w = rng.uniform(0.5, 1.5, size=N_CUT[name])
        coef = twosd_ref.Coefficients(sp2)
        pos = list(sto.indep.keys())
        deltas = [twosd_ref.delta_coefficients(coef, list(zip(pos, v))) for v in vals_c]
        a, b, wm, mv, ma = twosd_ref.build_sasa_cut(coef, deltas, w, x, Vset, tie_rel=0.0)
        np.savez_compressed(os.path.join(HERE, f"cut_{name}.npz"), x=x, values=vals_c, rows=rows, w=w,
                            V=Vset.matrix(sp2.W.shape[0]), alpha=a, beta=b, weight_mark=wm, max_val=mv,
                            max_arg=ma)
        print(name, "EV", evobj, "|V|", len(Vset), "alpha", a)
    with open(os.path.join(HERE, "ev_x.json"), "w") as f:
        json.dump(ev, f, indent=1)


if __name__ == "__main__":
    main()

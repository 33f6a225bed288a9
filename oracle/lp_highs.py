"""Second-stage LP via HiGHS (oracle; TEST INFRASTRUCTURE ONLY -- see oracle/__init__.py).

Restates ``solve_problem!`` (src/smps/smps_routines.jl:50-62): instantiate the scenario,
fix x, solve  min q'y  s.t.  W y {>=,<=,==} r_w - T_w x,  lb <= y <= ub,
and return (obj, y, pi) with pi in JuMP's dual convention for a MIN problem
(>= rows pi >= 0, <= rows pi <= 0, == rows free; pi = d obj / d rhs).

The reference uses GLPK 5.0.1 (Manifest.toml); GLPK is not available here, so
HiGHS (scipy 1.15.3, dual simplex, presolve off) stands in.  The optimal objective is
unique; the dual vertex is solver dependent on degenerate LPs.
Also: ``solve_ev`` solves the expected-value problem (stage 1 + stage 2 at the
mean scenario) to produce a first-stage x used by configs and fixtures.
"""
from __future__ import annotations

import numpy as np
from scipy.optimize import linprog


def _split(senses, W, b):
    G = [i for i, s in enumerate(senses) if s == 'G']
    L = [i for i, s in enumerate(senses) if s == 'L']
    E = [i for i, s in enumerate(senses) if s == 'E']
    A_ub = np.vstack([-W[G], W[L]]) if (G or L) else None
    b_ub = np.concatenate([-b[G], b[L]]) if (G or L) else None
    A_eq = W[E] if E else None
    b_eq = b[E] if E else None
    return G, L, E, A_ub, b_ub, A_eq, b_eq


def solve_rhs(sp, b, method="highs-ds"):
    """Solve min q'y s.t. W y (senses) b, bounds of sp.  Returns (status, obj, y, pi)."""
    G, L, E, A_ub, b_ub, A_eq, b_eq = _split(sp.senses, sp.W, b)
    bounds = list(zip(sp.cur_lb, [None if np.isinf(u) else u for u in sp.cur_ub]))
    res = linprog(sp.q, A_ub=A_ub, b_ub=b_ub, A_eq=A_eq, b_eq=b_eq, bounds=bounds,
                  method=method, options={"presolve": False})
    if res.status != 0:
        return res.status, np.nan, None, None
    pi = np.zeros(len(sp.senses))
    if G or L:
        mub = res.ineqlin.marginals
        pi[G] = -mub[:len(G)]
        pi[L] = mub[len(G):]
    if E:
        pi[E] = res.eqlin.marginals
    return 0, float(res.fun), res.x, pi


def solve_problem(sp, x, scenario_rhs):
    """solve_problem!(sp, x, omega) for RHS-only scenarios: scenario_rhs is the full
    stage-2 rhs vector r_w."""
    b = np.asarray(scenario_rhs, dtype=np.float64) - sp.T @ np.asarray(x, dtype=np.float64)
    return solve_rhs(sp, b)


def sto_mean_rhs(sp, sto):
    """r with every random RHS element replaced by its mean (DISCRETE: sum p v;
    NORMAL: mean; UNIFORM: (a+b)/2)."""
    r = sp.r.copy()
    rows = {n: i for i, n in enumerate(sp.row_names)}
    for (col, row), dist in sto.indep.items():
        if col not in ("RHS", "rhs"):
            continue
        if dist[0] == "DISCRETE":
            mu = float(np.dot(dist[1], dist[2]))
        elif dist[0] == "NORMAL":
            mu = dist[1]
        else:
            mu = 0.5 * (dist[1] + dist[2])
        r[rows[row]] = mu
    return r


def solve_ev(sp1, sp2, r2):
    """Extensive form with one scenario (rhs r2): min c'x + q'y, stage-1 rows, stage-2
    rows T x + W y (senses) r2.  Returns (obj, x)."""
    n1, n2 = sp1.W.shape[1], sp2.W.shape[1]
    m1, m2 = sp1.W.shape[0], sp2.W.shape[0]
    A = np.zeros((m1 + m2, n1 + n2))
    A[:m1, :n1] = sp1.W
    A[m1:, :n1] = sp2.T
    A[m1:, n1:] = sp2.W
    b = np.concatenate([sp1.r, r2])
    senses = list(sp1.senses) + list(sp2.senses)
    G, L, E, A_ub, b_ub, A_eq, b_eq = _split(senses, A, b)
    lb = np.concatenate([sp1.cur_lb, sp2.cur_lb])
    ub = np.concatenate([sp1.cur_ub, sp2.cur_ub])
    bounds = list(zip([None if np.isinf(l) else l for l in lb],
                      [None if np.isinf(u) else u for u in ub]))
    c = np.concatenate([sp1.q, sp2.q])
    res = linprog(c, A_ub=A_ub, b_ub=b_ub, A_eq=A_eq, b_eq=b_eq, bounds=bounds,
                  method="highs")
    assert res.status == 0, res.message
    return float(res.fun), res.x[:n1]


def extensive_form(sp1, sp2, scenario_rhs, probs=None):
    """all_in_one (src/crash.jl:18-72) via HiGHS: min c'x + sum_s p_s q'y_s, stage-1 rows,
    per scenario T x + W y_s (senses) r_s.  Returns the optimal objective."""
    S = len(scenario_rhs)
    probs = [1.0 / S] * S if probs is None else list(probs)
    n1, n2 = sp1.W.shape[1], sp2.W.shape[1]
    m1, m2 = sp1.W.shape[0], sp2.W.shape[0]
    A = np.zeros((m1 + S * m2, n1 + S * n2))
    A[:m1, :n1] = sp1.W
    for s in range(S):
        A[m1 + s * m2:m1 + (s + 1) * m2, :n1] = sp2.T
        A[m1 + s * m2:m1 + (s + 1) * m2, n1 + s * n2:n1 + (s + 1) * n2] = sp2.W
    b = np.concatenate([sp1.r] + [np.asarray(r, dtype=np.float64) for r in scenario_rhs])
    senses = list(sp1.senses) + list(sp2.senses) * S
    G, L, E, A_ub, b_ub, A_eq, b_eq = _split(senses, A, b)
    lb = np.concatenate([sp1.cur_lb] + [sp2.cur_lb] * S)
    ub = np.concatenate([sp1.cur_ub] + [sp2.cur_ub] * S)
    bounds = list(zip([None if np.isinf(l) else l for l in lb],
                      [None if np.isinf(u) else u for u in ub]))
    c = np.concatenate([sp1.q] + [p * sp2.q for p in probs])
    res = linprog(c, A_ub=A_ub, b_ub=b_ub, A_eq=A_eq, b_eq=b_eq, bounds=bounds, method="highs")
    assert res.status == 0, res.message
    return float(res.fun)

"""Oracle pinned by the committed golden fixtures (HiGHS duals / reference-order cuts,
tests/golden/make_golden.py) and self-consistency between its Python and C halves."""
import json
import os

import numpy as np
import pytest

from oracle import cpu, lp_highs, twosd_ref
from tests import instances as I

G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
NAMES = ["lands", "newsvendor", "transship", "ssn", "storm"]


def _lp_fixture(name):
    z = np.load(os.path.join(G, f"lp_{name}.npz"))
    return z["x"], z["values"], z["rows"], z["obj"], z["pi"]


@pytest.mark.parametrize("name", NAMES)
def test_highs_fixture_reproducible(name):
    """Re-solving the fixture scenarios with HiGHS gives the stored objective (unique) and a
    dual that certifies it (strong duality)."""
    x, vals, rows, obj, pi = _lp_fixture(name)
    sp = I.load(name)["osp2"]
    for v, o, p in zip(vals[:4], obj, pi):
        r = sp.r.copy(); r[rows] = v
        st, o2, _, p2 = lp_highs.solve_problem(sp, x, r)
        assert st == 0 and o2 == pytest.approx(o, rel=1e-9, abs=1e-9)
        b = r - sp.T @ x
        assert p @ b == pytest.approx(o, rel=1e-9, abs=1e-7)


@pytest.mark.parametrize("name", NAMES)
def test_c_dual_simplex_vs_highs_fixture(name):
    """The oracle C dual simplex (warm start from its own slack-basis solve of the mean
    scenario) reproduces the golden HiGHS objectives."""
    x, vals, rows, obj, pi = _lp_fixture(name)
    sp = I.load(name)["osp2"]
    lp = cpu.CpuLP(sp.W, sp.q, sp.senses)
    rmean = lp_highs.sto_mean_rhs(sp, I.load(name)["osto"])
    st, _, head, _ = lp.solve_from_slack(rmean - sp.T @ x)
    assert st == 0
    assert lp.set_basis(head) <= 1e-9
    o, p, _, s, _ = lp.solve_batch(rows.astype(np.int32), sp.r - sp.T @ x, vals - sp.r[rows], nthreads=1)
    assert (s == 0).all()
    np.testing.assert_allclose(o, obj, rtol=1e-9, atol=1e-8)
    for k in range(len(o)):
        b = sp.r - sp.T @ x
        b[rows] += vals[k] - sp.r[rows]
        assert p[k] @ b == pytest.approx(o[k], rel=1e-9, abs=1e-8)


@pytest.mark.parametrize("name", NAMES)
def test_cut_fixture(name):
    """Reference-order build_sasa_cut (Python restatement and C port) vs the golden cut."""
    z = np.load(os.path.join(G, f"cut_{name}.npz"))
    sp = I.load(name)["osp2"]
    coef = twosd_ref.Coefficients(sp)
    pos = list(I.load(name)["osto"].indep.keys())
    deltas = [twosd_ref.delta_coefficients(coef, list(zip(pos, v))) for v in z["values"]]
    V = twosd_ref.DualVertexSet(list(z["V"]))
    a, b, wm, mv, ma = twosd_ref.build_sasa_cut(coef, deltas, z["w"], z["x"], V)
    assert a == pytest.approx(float(z["alpha"]), rel=1e-12)
    np.testing.assert_allclose(b, z["beta"], rtol=1e-12, atol=1e-9)
    assert (ma == z["max_arg"]).all()
    a2, b2, mv2, ma2 = cpu.build_cut(sp.r, sp.T, z["x"], z["V"], z["rows"].astype(np.int32),
                                     z["values"] - sp.r[z["rows"]], z["w"], tie_rel=0.0, nthreads=1)
    assert a2 == pytest.approx(float(z["alpha"]), rel=1e-10)
    np.testing.assert_allclose(b2, z["beta"], rtol=1e-10, atol=1e-8)
    assert (ma2 == z["max_arg"]).all()
    np.testing.assert_allclose(mv2, z["max_val"], rtol=1e-10, atol=1e-8)


def test_ev_fixture():
    with open(os.path.join(G, "ev_x.json")) as f:
        ev = json.load(f)
    assert ev["storm"]["ev_obj"] == pytest.approx(1.5459266e7, rel=1e-7)     # SURVEY.md §8 d (C4)
    assert ev["lands"]["ev_obj"] == pytest.approx(378.667, rel=1e-5)

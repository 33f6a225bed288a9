"""Host master side (no GPU): the extensive form all_in_one against the
reference KAT (crash_test.jl:21-37: lands, 3 scenarios, p = (.3, .4, .3) -> 381.8533333),
the dense QP interior point against scipy (LP via HiGHS, KKT conditions for QPs), the
quad-scalar schedules (quad_scalar.jl) and the first-stage feasibility check (prob.jl)."""
import numpy as np
import pytest

from tests import instances as I


def _lands():
    from sqlp_amd import smps
    inst = I.load("lands")
    sp1 = smps.get_smps_stage_template(inst["cor"], inst["tim"], 1)
    return sp1, inst["sp2"]


def test_all_in_one_lands_kat():
    from sqlp_amd import master
    sp1, sp2 = _lands()
    row = sp2.stage_constraints.index("S2C5")
    rhs = []
    for v in (3.0, 5.0, 7.0):
        r = sp2.r.copy(); r[row] = v; rhs.append(r)
    obj, x, ys = master.all_in_one(sp1, sp2, rhs, [0.3, 0.4, 0.3])
    assert obj == pytest.approx(381.8533333, rel=1e-9)          # crash_test.jl:37
    assert len(ys) == 3 and all(len(y) == len(sp2.current_stage_vars) for y in ys)
    assert master.check_first_stage_feasible(sp1, x, tol=1e-8)
    # every scenario block is feasible with its own rhs
    W, T = sp2.dense_W(), sp2.dense_T()
    for r, y in zip(rhs, ys):
        res = W @ y + T @ x - r
        for i, s in enumerate(sp2.sense):
            if s == "G":
                assert res[i] >= -1e-7
            elif s == "L":
                assert res[i] <= 1e-7
            else:
                assert abs(res[i]) <= 1e-7


def test_all_in_one_matches_highs_extensive_form():
    """ssn-free check on transship: the extensive form over 4 sampled scenarios equals the
    oracle's HiGHS solve of the same deterministic equivalent."""
    from oracle import lp_highs
    from sqlp_amd import master, smps
    inst = I.load("transship")
    sp1 = smps.get_smps_stage_template(inst["cor"], inst["tim"], 1)
    sp2 = inst["sp2"]
    pos, rows, cols = smps.scenario_positions(sp2, inst["sto"])
    vals = I.sample("transship", 4, 5)
    rhs = []
    for v in vals:
        r = sp2.r.copy(); r[rows] = v; rhs.append(r)
    obj, x, _ = master.all_in_one(sp1, sp2, rhs)
    ref = lp_highs.extensive_form(I.load("transship")["osp1"], I.load("transship")["osp2"], rhs)
    assert obj == pytest.approx(ref, rel=1e-8)


def test_qp_solve_lp_matches_highs():
    from scipy.optimize import linprog
    from sqlp_amd import master
    rng = np.random.default_rng(0)
    for _ in range(5):
        n, me, mi = 12, 3, 10
        A = rng.normal(size=(me, n))
        x0 = rng.uniform(0.5, 1.5, size=n)
        b = A @ x0
        G = rng.normal(size=(mi, n))
        h = G @ x0 + rng.uniform(0.1, 1.0, size=mi)
        g = rng.normal(size=n)
        lo, hi = np.zeros(n), np.full(n, 3.0)
        Gb, hb = master._bound_rows(lo, hi, n)
        res = master.qp_solve(np.zeros(n), g, A, b, np.vstack([G, Gb]), np.concatenate([h, hb]))
        ref = linprog(g, A_ub=G, b_ub=h, A_eq=A, b_eq=b, bounds=list(zip(lo, hi)), method="highs")
        assert res.status == master.OPTIMAL and ref.status == 0
        assert res.obj == pytest.approx(ref.fun, rel=1e-8, abs=1e-8)


def test_qp_solve_kkt():
    """Strictly convex in x, linear in an epigraph variable (the master's shape): KKT holds."""
    from sqlp_amd import master
    rng = np.random.default_rng(1)
    n1 = 6
    cuts = rng.normal(size=(8, n1))
    alphas = rng.normal(size=8)
    # z = [x, eta]; min 0.5 rho |x - c|^2 + eta, eta >= a_j + b_j' x, x in [-2, 2]
    rho, c = 0.7, rng.normal(size=n1)
    H = np.concatenate([np.full(n1, rho), [0.0]])
    g = np.concatenate([-rho * c, [1.0]])
    G = np.hstack([cuts, -np.ones((8, 1))])
    h = -alphas
    Gb, hb = master._bound_rows(np.full(n1, -2.0), np.full(n1, 2.0), n1 + 1)
    GG, hh = np.vstack([G, Gb]), np.concatenate([h, hb])
    res = master.qp_solve(H, g, None, None, GG, hh)
    assert res.status == master.OPTIMAL
    z, lam = res.z, res.lam
    assert (GG @ z <= hh + 1e-8).all() and (lam >= -1e-10).all()
    np.testing.assert_allclose(H * z + g + GG.T @ lam, 0.0, atol=1e-7)
    assert abs(lam @ (GG @ z - hh)) <= 1e-7
    assert lam[:8].sum() == pytest.approx(1.0, rel=1e-7)        # d/d eta: sum of cut multipliers = 1


def test_quad_scalar_schedules():
    from sqlp_amd import master
    from sqlp_amd.twosd import sdImprovementInfo

    class Cell:
        pass
    cell = Cell()
    cell.ext = {}
    cell.x_incumbent = np.zeros(2)
    cell.x_candidate = np.array([1.0, 1.0])
    assert master.ConstantQuadScalarSchedule(0.1)(cell) == 0.1
    sched = master.AdaptiveQuadScalarSchedule()
    with pytest.raises(AssertionError):
        sched(cell)
    cell.ext["quad_scalar"] = 1.0
    cell.improvement_info = sdImprovementInfo(0, 0, 0, False)
    assert sched(cell) == pytest.approx(1.0 / 0.95)             # not improved: / R2 (quad_scalar.jl:63)
    cell.improvement_info = sdImprovementInfo(0, 0, 0, True)
    cell.x_candidate = np.array([3.0, 3.0])                     # normDk = 18 >= R3 * 2
    assert sched(cell) == pytest.approx(1.0 / 0.95 * 0.95 * 2.0 * 2.0 / 18.0)
    assert cell.ext["normDk_1"] == 18.0


def test_check_first_stage_feasible():
    from sqlp_amd import master
    sp1, _ = _lands()
    assert master.check_first_stage_feasible(sp1, np.array([3.0, 3.0, 3.0, 3.0]))
    assert not master.check_first_stage_feasible(sp1, np.zeros(4))        # sum x >= 12 violated
    assert not master.check_first_stage_feasible(sp1, np.array([-1.0, 5.0, 5.0, 5.0]))


def test_degenerate_master_multipliers_are_central():
    """Parity note for cut removal (algorithm.jl:57-72): with two identical cuts tight
    at the master optimum the dual is not unique.  The host IPM returns the central split
    (each row half of the multiplier one cut alone gets), where a simplex-type solver (the
    reference's CPLEX / GLPK) returns a vertex (all on one row).  The sum is what is unique, and
    it is what this asserts; which duplicate a vertex solver keeps is solver-dependent, so this
    part of the trajectory is unpinned."""
    from sqlp_amd import master
    # min 1/2 x^2 - 1/2 x + eta  s.t.  eta >= 2 - x (twice), eta >= 0, 0 <= x <= 10:
    # x* = 1.5, eta* = 0.5, only the cut is tight (multiplier 1)
    H = np.array([1.0, 0.0])
    g = np.array([-0.5, 1.0])
    G = np.array([[-1.0, -1.0], [-1.0, -1.0], [0.0, -1.0], [-1.0, 0.0], [1.0, 0.0]])
    h = np.array([-2.0, -2.0, 0.0, 0.0, 10.0])
    one = master.qp_solve(H, g, None, None, np.delete(G, 1, axis=0), np.delete(h, 1))
    two = master.qp_solve(H, g, None, None, G, h)
    assert one.status == two.status == master.OPTIMAL
    np.testing.assert_allclose(two.z, [1.5, 0.5], atol=1e-7)
    np.testing.assert_allclose(one.z, [1.5, 0.5], atol=1e-7)
    lam1, lam2 = one.lam[0], two.lam[:2]
    assert lam1 == pytest.approx(1.0, rel=1e-6)
    assert lam2.sum() == pytest.approx(lam1, rel=1e-6)
    assert lam2[0] == pytest.approx(lam2[1], rel=1e-6)        # central: split evenly

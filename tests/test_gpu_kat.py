"""The reference's lands known-answer tests, run through the GPU path (C ABI)."""
import numpy as np
import pytest

from tests import instances as I

pytestmark = pytest.mark.gpu

X1 = np.array([3.0, 3, 3, 3])
X2 = np.array([2.0, 4, 2, 6])


def _ctx():
    from sqlp_amd import smps, twosd
    inst = I.load("lands")
    ctx = twosd.SDContext(inst["sp2"], inst["sto"])
    ctx.compute_basis(I.x_ev("lands"), smps.mean_values(inst["sto"]))
    return ctx


def _sc(v):
    return [(("RHS", "S2C5"), v)]


def test_subgradient_kat():
    # test/sgd_example.jl:28, test/sd_test.jl:102
    from sqlp_amd import twosd
    ctx = _ctx()
    obj, y, pi = twosd.solve_problem(ctx, np.array([2.0, 3, 4, 5]), _sc(7.0))
    T = ctx.sp2.dense_T()
    assert (-(T.T @ pi)).tolist() == [-11.0, -6.0, -19.0, 0.0]


def test_strong_duality_kat():
    # test/sd_test.jl:45-65: eval_dual(coef, delta, x, dual) == objective
    from sqlp_amd import twosd
    ctx = _ctx()
    sp = I.load("lands")["osp2"]
    for v in (5.0, 3.0, 7.0):
        obj, y, pi = twosd.solve_problem(ctx, X1, _sc(v))
        r = sp.r.copy(); r[sp.row_names.index("S2C5")] = v
        assert abs(pi @ (r - sp.T @ X1) - obj) <= 1e-12 * (1 + abs(obj))


def test_vertex_count_and_argmax_kat():
    # test/sd_test.jl:75-94
    from sqlp_amd import twosd
    ctx = _ctx()
    V = twosd.sdDualVertexSet(ctx)
    scen = [5.0, 5.0, 3.0, 7.0]
    for v in scen:
        twosd.push(V, twosd.solve_problem(ctx, X1, _sc(v))[2])
    assert len(V) == 3
    epi = twosd.sdEpigraph(ctx, 1.0, 0.0)
    for v in scen:
        twosd.add_scenario(epi, _sc(v), 1.0)
    val, arg = twosd.argmax_procedure(epi, X2, V, tie_rel=0.0)
    for v, mv in zip(scen, val):
        obj = twosd.solve_problem(ctx, X2, _sc(v))[0]
        assert abs(mv - obj) <= 1e-12 * (1 + abs(obj))


def test_build_sasa_cut_kat():
    # test/sd_test.jl:209-235
    from sqlp_amd import twosd
    ctx = _ctx()
    sp = I.load("lands")["osp2"]
    d5 = twosd.solve_problem(ctx, X1, _sc(5.0))[2]
    d3 = twosd.solve_problem(ctx, X1, _sc(3.0))[2]
    V = twosd.sdDualVertexSet(ctx, [d5, d3])
    epi = twosd.sdEpigraph(ctx, 0.5, 100.0)
    twosd.add_scenario(epi, _sc(3.0), 1.5)
    twosd.add_scenario(epi, _sc(7.0), 0.5)
    x = np.array([2.0, 3, 4, 5])
    cut = twosd.build_sasa_cut(epi, x, V, tie_rel=0.0)
    _, arg = twosd.argmax_procedure(epi, x, V, tie_rel=0.0)
    Vm = V.matrix()
    row = sp.row_names.index("S2C5")
    r1 = sp.r.copy(); r1[row] = 3.0
    r2 = sp.r.copy(); r2[row] = 7.0
    dA, dB = Vm[arg[0]], Vm[arg[1]]
    assert cut.alpha == pytest.approx(1.5 / 2.0 * dA @ r1 + 0.5 / 2.0 * dB @ r2, rel=1e-13)
    np.testing.assert_allclose(cut.beta, 1.5 / 2.0 * -(sp.T.T @ dA) + 0.5 / 2.0 * -(sp.T.T @ dB), rtol=1e-13)
    assert cut.weight_mark == 2.0
    assert epi.total_scenario_weight == 2.0


def test_sd_iteration_hot_path():
    """sd_iteration! data-parallel segment on 2 epigraphs: vertex order cand/inc interleaved,
    cuts appended per epigraph, incumbent cut replaced (algorithm.jl:45-55, 79-85)."""
    from sqlp_amd import twosd
    ctx = _ctx()
    V = twosd.sdDualVertexSet(ctx)
    epis = [twosd.sdEpigraph(ctx, 0.5, 0.0) for _ in range(2)]
    xc, xi = I.x_ev("lands"), X1
    for it in range(3):
        vals = [I.sample("lands", 1, 100 * it + e) for e in range(2)]
        twosd.sd_iteration_hot_path(epis, vals, xc, xi, V)
    assert all(len(e.cuts) == 3 and e.incumbent_cut is not None for e in epis)
    assert all(e.num_scenarios == 3 for e in epis)
    assert 1 <= len(V) <= 12

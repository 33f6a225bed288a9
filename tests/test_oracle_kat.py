"""The oracle restatement pinned by the reference's own known-answer tests (lands).

Each test cites the reference test it reproduces (paths relative to yhz0/SQLP).  The LP is
solved by HiGHS (scipy) and by the oracle's C dual simplex; the reference used GLPK.
"""
import numpy as np
import pytest

from oracle import cpu, lp_highs, smps_ref, twosd_ref
from tests import instances as I

LANDS = I.DATA + "/lands"


@pytest.fixture(scope="module")
def lands():
    cor, tim, sto = smps_ref.load_instance(LANDS, "lands")
    return cor, tim, sto, smps_ref.stage_template(cor, tim, 1), smps_ref.stage_template(cor, tim, 2)


def test_smps_tokens_kat():
    # test/smps_tests.jl:5-20
    with open(LANDS + "/lands.cor") as f:
        tok = smps_ref.tokenize_cor(f.read().splitlines())
    d, rows = smps_ref.parse_row_tokens(tok["ROWS"])
    assert "".join(d) == "NGLLLLLGGG"
    assert rows == ["OBJ", "S1C1", "S1C2", "S2C1", "S2C2", "S2C3", "S2C4", "S2C5", "S2C6", "S2C7"]
    cols = smps_ref.parse_unique_columns(tok["COLUMNS"])
    assert cols == ["X1", "X2", "X3", "X4", "Y11", "Y21", "Y31", "Y41", "Y12", "Y22", "Y32", "Y42",
                    "Y13", "Y23", "Y33", "Y43"]
    M = smps_ref.parse_column_to_matrix(tok["COLUMNS"], rows, cols)
    assert np.count_nonzero(M) == 52                         # :23
    rhs = smps_ref.parse_rhs(tok["RHS"], rows)
    assert rhs.tolist() == [0., 12, 120, 0, 0, 0, 0, 0, 3, 2]  # :27
    lb, ub = smps_ref.parse_bounds(tok["BOUNDS"], cols)
    assert (lb == 0).all() and np.isinf(ub).all()             # :30-32


def test_smps_tim_sto_stage_kat(lands):
    cor, tim, sto, sp1, sp2 = lands
    # test/smps_tests.jl:36-38, 46-50, 55-58
    assert tim.problem_name == "LandS"
    assert tim.periods[0] == ("TIME1", "X1", "OBJ")
    assert tim.periods[1] == ("TIME2", "Y11", "S2C1")
    assert len(sp1.cur_names) == 4 and len(sp1.row_names) == 2
    assert len(sp2.last_names) + len(sp2.cur_names) == 16 and len(sp2.row_names) == 7
    assert sto.problem_name == "LandS"
    d = sto.indep[("RHS", "S2C5")]
    assert d[1] == [3.0, 5.0, 7.0] and d[2] == [0.3, 0.4, 0.3]


def test_dual_set_kat():
    # test/dual_set_test.jl:2-33
    v1, v2, v3 = [1., 2, 3], [1.0000000001, 2, 3], [4., 5, 6]
    v4, v5 = [4., 5, 6, 7], [3., 2, 1]
    h = twosd_ref.hash_dual_vector
    eq = lambda a, b: twosd_ref.dual_isequal(h(a), a, h(b), b)
    assert eq(v1, v2) and eq(v3, v3)
    assert not eq(v1, v3) and not eq(v3, v4) and not eq(v5, v1)
    V = twosd_ref.DualVertexSet()
    sizes = []
    for v in (v1, v2, v3, v4, v5):
        V.push(v)
        sizes.append(len(V))
    assert sizes == [1, 1, 2, 3, 4]
    assert len(twosd_ref.DualVertexSet([v1, v2, v3, v4, v5])) == 4
    assert len(list(twosd_ref.DualVertexSet([v1, v2, v3, v4, v5]))) == 4


def test_round16_semantics():
    # Julia round(x; base=2, sigdigits=16): keep 16 significant bits, ties to even
    r = twosd_ref.round16
    assert r(1.0) == 1.0 and r(0.0) == 0.0 and r(-3.5) == -3.5
    assert r(1.0 + 2.0 ** -20) == 1.0
    assert r(1.0 + 2.0 ** -15) == 1.0 + 2.0 ** -15
    assert r(1.0 + 2.0 ** -16) == 1.0                       # tie -> even
    assert r(1.0 + 3 * 2.0 ** -16) == 1.0 + 2.0 ** -14      # tie -> even (up)
    assert r(1.0000000001) == 1.0
    assert r(12345.678) == round(12345.678 * 2 ** 2) / 2 ** 2
    assert np.isinf(r(np.inf)) and np.isnan(r(np.nan))


def _kat_setup(lands):
    cor, tim, sto, sp1, sp2 = lands
    coef = twosd_ref.Coefficients(sp2)
    sc = lambda v: [(("RHS", "S2C5"), v)]
    return sp2, coef, sc


def test_delta_and_eval_dual_kat(lands):
    sp2, coef, sc = _kat_setup(lands)
    # test/sd_test.jl:19-23
    assert coef.row_lookup["S2C5"] == 4 and coef.col_lookup["X2"] == 1   # 0-based here
    with pytest.raises(KeyError):
        coef.col_lookup["Y11"]
    # sd_test.jl:36-41: template rhs S2C5 = 3 -> delta for 5 is 2
    coef3 = twosd_ref.Coefficients(sp2)
    coef3.rhs[coef3.row_lookup["S2C5"]] = 3.0
    dr, dT = twosd_ref.delta_coefficients(coef3, sc(5.0))
    assert dr[coef3.row_lookup["S2C5"]] == 2.0 and dT.sum() == 0.0
    with pytest.raises(KeyError):
        twosd_ref.delta_coefficients(coef3, [(("Y11", "S2C5"), 1.0)])
    # sd_test.jl:45-65: strong duality eval_dual == objective at x = [3,3,3,3]
    x = np.array([3.0, 3, 3, 3])
    for v in (5.0, 3.0):
        r = sp2.r.copy(); r[coef.row_lookup["S2C5"]] = v
        st, obj, y, pi = lp_highs.solve_problem(sp2, x, r)
        val = twosd_ref.eval_dual(coef3, twosd_ref.delta_coefficients(coef3, sc(v)), x, pi)
        assert abs(val - obj) <= 1e-12 * (1 + abs(obj))


def test_subgradient_kat(lands):
    # test/sgd_example.jl:27-28 and test/sd_test.jl:97-103
    sp2, coef, sc = _kat_setup(lands)
    x = np.array([2.0, 3, 4, 5])
    r = sp2.r.copy(); r[coef.row_lookup["S2C5"]] = 7.0
    st, obj, y, pi = lp_highs.solve_problem(sp2, x, r)
    assert (-(sp2.T.T @ pi)).tolist() == [-11.0, -6.0, -19.0, 0.0]
    # the C oracle from its own slack-basis solve
    lp = cpu.CpuLP(sp2.W, sp2.q, sp2.senses)
    st2, obj2, head, _ = lp.solve_from_slack(r - sp2.T @ x)
    lp.set_basis(head)
    o, p, _, s, _ = lp.solve_batch(np.array([4], dtype=np.int32), r - sp2.T @ x, np.zeros((1, 1)))
    assert s[0] == 0 and abs(o[0] - obj) < 1e-9
    assert (-(sp2.T.T @ p[0])).tolist() == [-11.0, -6.0, -19.0, 0.0]


def test_vertex_count_and_argmax_kat(lands):
    # test/sd_test.jl:75-94: 4 solves at x1 give |V| = 3; argmax at x2 equals the LP value
    sp2, coef, sc = _kat_setup(lands)
    x1, x2 = np.array([3.0, 3, 3, 3]), np.array([2.0, 4, 2, 6])
    scen = [5.0, 5.0, 3.0, 7.0]
    V = twosd_ref.DualVertexSet()
    row = coef.row_lookup["S2C5"]
    for v in scen:
        r = sp2.r.copy(); r[row] = v
        V.push(lp_highs.solve_problem(sp2, x1, r)[3])
    assert len(V) == 3
    deltas = [twosd_ref.delta_coefficients(coef, sc(v)) for v in scen]
    vals, args = twosd_ref.argmax_procedure(coef, deltas, x2, V)
    for v, mv in zip(scen, vals):
        r = sp2.r.copy(); r[row] = v
        obj = lp_highs.solve_problem(sp2, x2, r)[1]
        assert abs(mv - obj) <= 1e-9 * (1 + abs(obj))


def test_build_sasa_cut_kat(lands):
    # test/sd_test.jl:209-235 (weights 1.5 / 0.5, V = {dual(S2C5=5), dual(S2C5=3)} at x=[3,3,3,3])
    sp2, coef, sc = _kat_setup(lands)
    row = coef.row_lookup["S2C5"]
    x3 = np.array([3.0, 3, 3, 3])
    duals = []
    for v in (5.0, 3.0):
        r = sp2.r.copy(); r[row] = v
        duals.append(lp_highs.solve_problem(sp2, x3, r)[3])
    V = twosd_ref.DualVertexSet(duals)
    x = np.array([2.0, 3, 4, 5])
    deltas = [twosd_ref.delta_coefficients(coef, sc(3.0)), twosd_ref.delta_coefficients(coef, sc(7.0))]
    a, b, wm, mv, ma = twosd_ref.build_sasa_cut(coef, deltas, [1.5, 0.5], x, V)
    r1 = coef.rhs + deltas[0][0]
    r2 = coef.rhs + deltas[1][0]
    d1, d2 = V.data[ma[0]], V.data[ma[1]]
    assert a == pytest.approx(1.5 / 2.0 * d1 @ r1 + 0.5 / 2.0 * d2 @ r2, rel=1e-14)
    assert np.allclose(b, 1.5 / 2.0 * -(coef.transfer.T @ d1) + 0.5 / 2.0 * -(coef.transfer.T @ d2), rtol=1e-14)
    assert wm == 2.0


def test_evaluate_epigraph_kat():
    # test/sd_test.jl:166-194: cuts (1,[2..5],1), (6,[7..10],2), incumbent (11,[12..15],1)
    cut1, cut2 = (1.0, np.array([2.0, 3, 4, 5]), 1.0), (6.0, np.array([7.0, 8, 9, 10]), 2.0)
    inc = (11.0, np.array([12.0, 13, 14, 15]), 1.0)
    x = np.full(4, 10.0)
    assert 0.5 * twosd_ref.evaluate_epigraph([cut1, cut2], inc, x, 2.0, 0.0) == 551.0 * 0.5
    assert 0.5 * twosd_ref.evaluate_epigraph([cut1], None, x, 2.0, 100.0) == (141 / 2 + 100 / 2) * 0.5
    assert 0.5 * twosd_ref.evaluate_epigraph([cut1], None, np.full(4, -1.0), 2.0, 100.0) == 100.0 * 0.5
    # discounted rhs of add_cut_to_master! (sd_test.jl:184-187): 100*0.5 + 1.0*0.5
    assert twosd_ref.add_cut_discount(1.0, cut1[1], 0.5, 100.0)[0] == 50.5


def test_extensive_form_kat(lands):
    # test/crash_test.jl:21-37: lands with S2C5 in {3,5,7}, p = (.3,.4,.3) -> 381.8533333
    from scipy.optimize import linprog
    cor, tim, sto, sp1, sp2 = lands
    n1, n2 = sp1.W.shape[1], sp2.W.shape[1]
    m1, m2 = sp1.W.shape[0], sp2.W.shape[0]
    S = [3.0, 5.0, 7.0]
    p = [0.3, 0.4, 0.3]
    nv = n1 + len(S) * n2
    rows, b, sense = [], [], []
    for i in range(m1):
        a = np.zeros(nv); a[:n1] = sp1.W[i]; rows.append(a); b.append(sp1.r[i]); sense.append(sp1.senses[i])
    row5 = sp2.row_names.index("S2C5")
    for s, v in enumerate(S):
        r = sp2.r.copy(); r[row5] = v
        for i in range(m2):
            a = np.zeros(nv); a[:n1] = sp2.T[i]; a[n1 + s * n2:n1 + (s + 1) * n2] = sp2.W[i]
            rows.append(a); b.append(r[i]); sense.append(sp2.senses[i])
    A, b = np.array(rows), np.array(b)
    G = [i for i, t in enumerate(sense) if t == 'G']
    L = [i for i, t in enumerate(sense) if t == 'L']
    c = np.concatenate([sp1.q] + [p[s] * sp2.q for s in range(len(S))])
    res = linprog(c, A_ub=np.vstack([-A[G], A[L]]), b_ub=np.concatenate([-b[G], b[L]]), method="highs")
    assert res.fun == pytest.approx(381.8533333, abs=1e-6)


# ---- on-device sampler's oracle (oracle/sampler.c): Philox4x32-10 known answers ------------
# Random123 kat_vectors (Salmon et al., SC'11) for philox4x32 with 10 rounds.
PHILOX_KAT = [
    ([0, 0, 0, 0], [0, 0], [0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8]),
    ([0xffffffff] * 4, [0xffffffff] * 2, [0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd]),
    ([0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344], [0xa4093822, 0x299f31d0],
     [0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1]),
]


@pytest.mark.parametrize("ctr,key,expect", PHILOX_KAT)
def test_philox_kat(ctr, key, expect):
    from oracle import cpu
    assert list(cpu.philox4x32_10(ctr, key)) == expect


def test_sampler_oracle_distributions():
    """rand(rng, sto) transforms (smps_sto.jl:117-130): DiscreteNonParametric frequencies
    and sorted support, Normal(mean, sqrt(variance)), Uniform(left, right)."""
    from oracle import cpu
    from sqlp_amd.smps import spStoType, spSmpsPosition
    sto = spStoType("t", {})
    pa, pb, pc = spSmpsPosition("RHS", "A"), spSmpsPosition("RHS", "B"), spSmpsPosition("RHS", "C")
    sto.indep[pa] = ("DISCRETE", [7.0, 3.0, 5.0], [0.3, 0.3, 0.4])     # unsorted support
    sto.indep[pb] = ("NORMAL", 10.0, 4.0)                               # variance 4 -> sd 2
    sto.indep[pc] = ("UNIFORM", -1.0, 3.0)
    N = 200000
    d = cpu.sample_deltas(sto, [pa, pb, pc], [0.0, 0.0, 0.0], N, seed=12345)
    vals, cnt = np.unique(d[:, 0], return_counts=True)
    assert list(vals) == [3.0, 5.0, 7.0]
    np.testing.assert_allclose(cnt / N, [0.3, 0.4, 0.3], atol=0.005)   # probabilities follow the sorted support
    assert abs(d[:, 1].mean() - 10.0) < 0.02 and abs(d[:, 1].std() - 2.0) < 0.02
    assert d[:, 2].min() >= -1.0 and d[:, 2].max() < 3.0 and abs(d[:, 2].mean() - 1.0) < 0.01
    # a stream is a function of (seed, index, element): shards reproduce it
    d2 = np.vstack([cpu.sample_deltas(sto, [pa, pb, pc], [0.0] * 3, 1000, 12345, 0),
                    cpu.sample_deltas(sto, [pa, pb, pc], [0.0] * 3, 1000, 12345, 1000)])
    np.testing.assert_array_equal(d2, d[:2000])

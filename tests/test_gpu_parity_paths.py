"""GPU parity of the hot-path branches the SMPS instances never reach by themselves:

* random technology-matrix (T) elements: delta_coefficients' T branch (subprob.jl:115-117,
  dT[row, col] = val - T[row, col]) in the LP rhs b = (r + dr) - (T + dT) x and in the cut,
  beta = -sum_i p_i (T + dT_i)' pi_i (epigraph.jl:141), against oracle/twosd_ref.py and the
  C dual simplex;
* evaluate (smps_routines.jl:67-82) against the C oracle's in-order sum of (1/N) obj;
* the 1-based index path of the C ABI (Julia SparseMatrixCSC colptr / rowval);
* non-optimal scenarios: solve_problem! only logs @error for them (smps_routines.jl:54-57);
  here they surface as status[] = INFEASIBLE / ITER_LIMIT and TWOSD_E_LP, including a pool
  start retried from the primary basis.
All compute goes through libtwosd_hip.so; the oracle is only the checker."""
import numpy as np
import pytest

from tests import instances as I

pytestmark = pytest.mark.gpu


def _ctx(name, positions=None, index_base=0):
    from sqlp_amd import smps, twosd
    inst = I.load(name)
    ctx = twosd.SDContext(inst["sp2"], inst["sto"], positions=positions, index_base=index_base)
    x = I.x_ev(name)
    ctx.compute_basis(x, smps.mean_values(inst["sto"]) if positions is None else None)
    return ctx, x


# ---------------------------------------------------------------- random T elements
T_CASES = {
    # instance: extra positions (first-stage column, stage-2 row) and the sampling range; lands
    # keeps T[S2C1, X1] <= -1 so the EV capacity (12) still covers the largest demand (7 + 3 + 2)
    "lands": [(("X1", "S2C1"), (-1.3, -1.0)), (("X2", "S2C5"), (0.0, 0.4))],
    # transship's T entries sit in flow-balance equalities (initInv / finalInv = orderUp), so
    # any perturbation of one alone is infeasible (HiGHS agrees); ssn's capacity rows
    # LN* <= CAP* are not, and x_EV is nonzero on these two columns
    "ssn": [(("CAP2ZPZ", "LN2ZPZ"), (-1.2, -0.8)), (("CAPBUPP", "LNBUPP"), (-1.2, -0.8))],
}


def _t_scenarios(name, N, seed):
    """Values of the instance's own random elements plus the T elements of T_CASES."""
    inst = I.load(name)
    rng = np.random.default_rng(seed)
    base = I.sample(name, N, seed)
    extra = np.column_stack([rng.uniform(lo, hi, size=N) for _, (lo, hi) in T_CASES[name]])
    positions = list(inst["sto"].indep.keys()) + [p for p, _ in T_CASES[name]]
    return positions, np.hstack([base, extra])


def _oracle_rhs_deltas(sp, positions, vals, x):
    """rows + per-scenario rhs deltas of the oracle LP: dr for RHS entries, -(dT) x[col] for
    T entries (b = (r + dr) - (T + dT) x, instantiate! + fix(x))."""
    rows = np.array([sp.row_names.index(p[1]) for p in positions], dtype=np.int32)
    DR = np.empty_like(vals)
    for e, (col, row) in enumerate(positions):
        i = rows[e]
        if col in ("RHS", "rhs"):
            DR[:, e] = vals[:, e] - sp.r[i]
        else:
            j = sp.last_names.index(col)
            DR[:, e] = -(vals[:, e] - sp.T[i, j]) * x[j]
    return rows, DR


@pytest.mark.parametrize("name", ["lands", "ssn"])
def test_random_T_elements_lp_and_cut(name):
    from oracle import cpu, twosd_ref
    from sqlp_amd import twosd
    positions, vals = _t_scenarios(name, 160, seed=31)
    ctx, x = _ctx(name, positions=positions)
    assert (ctx.cols >= 0).sum() == len(T_CASES[name])
    sp = I.load(name)["osp2"]
    # LP: objectives equal the C dual simplex on b = (r + dr) - (T + dT) x; strong duality
    obj, _, pi, st = ctx.solve_values(x, vals, want_pi=True)
    assert (st == 0).all()
    rows, DR = _oracle_rhs_deltas(sp, positions, vals, x)
    lp = cpu.CpuLP(sp.W, sp.q, sp.senses)
    lp.set_basis(ctx.get_basis())
    o_obj, o_pi, _, o_st, _ = lp.solve_batch(rows, sp.r - sp.T @ x, DR, nthreads=4)
    assert (o_st == 0).all()
    np.testing.assert_allclose(obj, o_obj, rtol=1e-9, atol=1e-9)
    coef = twosd_ref.Coefficients(sp)
    deltas = [twosd_ref.delta_coefficients(coef, list(zip(positions, v))) for v in vals]
    for s in range(len(vals)):
        assert abs(twosd_ref.eval_dual(coef, deltas[s], x, pi[s]) - obj[s]) <= 1e-9 * (1 + abs(obj[s]))
    # cut: V from the LP duals; build_sasa_cut at a different x, random weights
    V = twosd.sdDualVertexSet(ctx)
    V.push_batch(pi)
    ov = twosd_ref.DualVertexSet(list(pi))
    assert len(V) == len(ov)
    np.testing.assert_array_equal(V.matrix(), ov.matrix())
    x2 = x * np.random.default_rng(4).uniform(0.8, 1.2, size=x.shape)
    w = np.random.default_rng(5).uniform(0.5, 1.5, size=len(vals))
    epi = twosd.sdEpigraph(ctx, 1.0, 0.0)
    twosd.add_scenarios(epi, vals, w)
    for xx in (x, x2):
        cut, mv, ma = twosd._build_cut(epi, xx, 0.0, want_argmax=True)
        a, b, wm, omv, oma = twosd_ref.build_sasa_cut(coef, deltas, w, xx, ov, tie_rel=0.0)
        assert cut.weight_mark == pytest.approx(wm, rel=1e-15)
        np.testing.assert_allclose(mv, omv, rtol=1e-10, atol=1e-9)
        Vm = ov.matrix()
        scores = np.array([[twosd_ref.eval_dual(coef, d, xx, p) for p in Vm] for d in deltas])
        top2 = np.sort(scores, axis=1)[:, -2:]
        clear = (top2[:, 1] - top2[:, 0]) > 1e-9 * (1 + np.abs(top2[:, 1]))
        assert (ma[clear] == oma[clear]).all()
        # the cut over the GPU's picks equals the reference formula (epigraph.jl:134-143)
        p = w / w.sum()
        a_g = sum(p[i] * float(Vm[ma[i]] @ (coef.rhs + deltas[i][0])) for i in range(len(vals)))
        b_g = sum(-p[i] * ((coef.transfer + deltas[i][1]).T @ Vm[ma[i]]) for i in range(len(vals)))
        assert cut.alpha == pytest.approx(a_g, rel=1e-9, abs=1e-9)
        np.testing.assert_allclose(cut.beta, b_g, rtol=1e-9, atol=1e-9 * (1 + np.abs(b_g).max()))
        if clear.all():
            assert cut.alpha == pytest.approx(a, rel=1e-8, abs=1e-8)
            np.testing.assert_allclose(cut.beta, b, rtol=1e-8, atol=1e-8 * (1 + np.abs(b).max()))


def test_random_T_element_unknown_column_raises():
    """delta_coefficients' KeyError for a column that is not a first-stage variable
    (subprob.jl:116) -> KeyError in the host layer before any device call."""
    from sqlp_amd import twosd
    inst = I.load("lands")
    with pytest.raises(KeyError):
        twosd.SDContext(inst["sp2"], inst["sto"], positions=[("Y11", "S2C1")])


# ---------------------------------------------------------------- evaluate vs the oracle
@pytest.mark.parametrize("name,N", [("lands", 20000), ("transship", 20000), ("storm", 8192)])
def test_evaluate_sampled_matches_oracle_sum(name, N):
    """evaluate(sp1, sp2, sto, x; N) on the device-drawn stream == c'x + sum_w (1/N) obj_w with
    obj from the C dual simplex on the same stream, summed in sample order
    (smps_routines.jl:76-80)."""
    from oracle import cpu
    from sqlp_amd import twosd
    ctx, x = _ctx(name)
    ctx.set_distributions(I.load(name)["sto"])
    c1 = np.linspace(1.0, 2.0, len(x))
    seed = 777
    val = twosd.evaluate_sampled(ctx, c1, x, N, seed)
    sp = I.load(name)["osp2"]
    deltas = cpu.sample_deltas(I.load(name)["sto"], ctx.positions, ctx.template_values, N, seed)
    lp = cpu.CpuLP(sp.W, sp.q, sp.senses)
    lp.set_basis(ctx.get_basis())
    o_obj, _, _, o_st, _ = lp.solve_batch(ctx.rows, sp.r - sp.T @ x, deltas, nthreads=8)
    assert (o_st == 0).all()
    s2 = 0.0
    for o in o_obj:
        s2 += 1.0 / N * o
    ref = float(c1 @ x) + s2
    assert abs(val - ref) <= 1e-10 * (1 + abs(ref)), (val, ref)


# ---------------------------------------------------------------- 1-based indices (Julia)
@pytest.mark.parametrize("name", ["lands", "ssn"])
def test_index_base_one_matches_base_zero(name):
    """twosd_set_template / twosd_set_random_positions with Int64 CSC arrays shifted to
    1-based (colptr + 1, rowval + 1, rows / cols + 1) give bit-identical LP and cut results."""
    from sqlp_amd import twosd
    positions, vals = _t_scenarios(name, 96, seed=8)
    out = []
    for ib in (0, 1):
        ctx, x = _ctx(name, positions=positions, index_base=ib)
        obj, _, pi, st = ctx.solve_values(x, vals, want_pi=True)
        assert (st == 0).all()
        V = twosd.sdDualVertexSet(ctx)
        V.push_batch(pi)
        epi = twosd.sdEpigraph(ctx, 1.0, 0.0)
        twosd.add_scenarios(epi, vals)
        cut = twosd.build_sasa_cut(epi, x, V, tie_rel=0.0)
        out.append((obj, pi, V.matrix(), cut.alpha, cut.beta, ctx.get_basis()))
    for a, b in zip(out[0], out[1]):
        np.testing.assert_array_equal(a, b)


def test_index_base_out_of_range_rejected():
    from sqlp_amd import twosd
    from sqlp_amd._lib import TwoSDError
    inst = I.load("lands")
    ctx = twosd.SDContext(inst["sp2"], inst["sto"], index_base=1)
    rows = np.array([0], dtype=np.int32)              # row 0 is out of range when 1-based
    cols = np.array([-1], dtype=np.int32)
    from sqlp_amd._lib import ptr
    with pytest.raises(TwoSDError):
        from sqlp_amd._lib import check
        check(ctx.lib.twosd_set_random_positions(ctx.h, 1, ptr(rows), ptr(cols), 1))


# ---------------------------------------------------------------- non-optimal scenarios
def test_infeasible_scenario_status():
    """lands has no recourse slack: demand S2C5 far above the installed capacity is
    infeasible.  The LP kernel reports it in status[] (dual ray: no entering column) and the
    batch call returns TWOSD_E_LP; the other scenarios of the batch are unaffected."""
    from sqlp_amd import twosd
    from sqlp_amd._lib import LP_INFEASIBLE, TwoSDError
    ctx, x = _ctx("lands")
    vals = np.array([[5.0], [1000.0], [3.0], [7.0], [2000.0]])
    obj, _, pi, st = ctx.solve_values(x, vals, want_pi=True, raise_on_status=False)
    assert st.tolist() == [0, LP_INFEASIBLE, 0, 0, LP_INFEASIBLE]
    assert np.isnan(pi[1]).all() and np.isnan(pi[4]).all()
    ok = ctx.solve_values(x, vals[[0, 2, 3]], want_pi=True)
    np.testing.assert_array_equal(obj[[0, 2, 3]], ok[0])
    with pytest.raises(TwoSDError) as e:
        ctx.solve_values(x, vals)
    assert e.value.code == -4
    # the device push path refuses to push the junk dual of a non-optimal scenario
    epi = twosd.sdEpigraph(ctx, 1.0, 0.0)
    twosd.add_scenarios(epi, vals)
    with pytest.raises(TwoSDError):
        twosd.solve_push(epi, x, 0, len(vals))


def test_iteration_limit_status_and_pool_retry(monkeypatch):
    """A pivot cap (TWOSD_KMAX, read at context creation) below what storm scenarios need
    ends them with status ITER_LIMIT.  With a basis pool, a pool start that hits the cap is
    retried from the primary basis (so the pool never changes which scenarios solve): the
    recorded pick of such a scenario is 0 (the primary basis), and with a cap that the
    primary start can meet, the objectives equal the uncapped run."""
    from sqlp_amd import twosd
    from sqlp_amd._lib import LP_ITER_LIMIT
    vals = I.sample("storm", 256, seed=3)
    ctx, x = _ctx("storm")
    ref, _, _, st0 = ctx.solve_values(x, vals)
    assert (st0 == 0).all()
    piv_primary = ctx.lp_stats()[1]                     # max pivots from the primary basis
    monkeypatch.setenv("TWOSD_KMAX", "2")
    capped, _ = _ctx("storm")
    obj, _, _, st = capped.solve_values(x, vals, raise_on_status=False)
    assert (st == LP_ITER_LIMIT).sum() > 0
    np.testing.assert_array_equal(obj[st == 0], ref[st == 0])
    # pool + a cap between the pool's and the primary basis' needs: every pool start that
    # hits the cap is retried from the primary basis and solves
    monkeypatch.setenv("TWOSD_KMAX", str(piv_primary))
    pooled, _ = _ctx("storm")
    tr = twosd.sdEpigraph(pooled, 1.0, 0.0)
    twosd.add_scenarios(tr, I.sample("storm", 2048, seed=11))
    assert pooled.pool_build(tr, x, 0, 2048, 16) > 1
    obj2, _, _, st2 = pooled.solve_values(x, vals)
    assert (st2 == 0).all()
    np.testing.assert_allclose(obj2, ref, rtol=1e-9, atol=1e-9)
    monkeypatch.setenv("TWOSD_KMAX", "1")
    tiny, _ = _ctx("storm")
    tr = twosd.sdEpigraph(tiny, 1.0, 0.0)
    twosd.add_scenarios(tr, I.sample("storm", 2048, seed=11))
    monkeypatch.delenv("TWOSD_KMAX")
    tiny.pool_add_basis(pooled.pool_get(1))
    obj3, _, _, st3 = tiny.solve_values(x, vals, raise_on_status=False)
    picks = tiny.last_pool_picks(len(vals))
    failed = st3 == LP_ITER_LIMIT
    assert failed.any()
    assert (picks[failed] == 0).all()                  # retried from the primary basis
    retried = tiny.lp_counts()[1]                      # pool starts solved again from the primary basis
    assert 0 < retried <= len(vals)


@pytest.mark.parametrize("name", ["storm", "transship"])
def test_last_objective_is_weighted_sum(name):
    """twosd_last_objective: the batch's sum_s w_s obj_s and sum_s w_s (add_scenario! weights), a
    fixed-order device reduction -- the same bits for solve_batch and solve_push of the same
    batch, and the host sum of the returned objectives to rounding."""
    from sqlp_amd import twosd
    ctx, x = _ctx(name)
    N = 3000
    vals = I.sample(name, N, seed=23)
    w = np.random.default_rng(4).uniform(0.5, 2.0, size=N)
    epi = twosd.sdEpigraph(ctx, 1.0, 0.0)
    twosd.add_scenarios(epi, vals, w)
    obj, _, _, st = twosd.solve_batch(epi, x, 0, N, want_pi=False)
    assert (st == 0).all()
    a, b = ctx.last_objective()
    assert b == pytest.approx(w.sum(), rel=1e-14)
    assert a == pytest.approx(float(np.dot(w, obj)), rel=1e-12)
    twosd.sdDualVertexSet(ctx)
    twosd.solve_push(epi, x, 0, N, want_obj=False)
    assert ctx.last_objective() == (a, b)
    # a sub-range: weights first..first+count
    twosd.solve_batch(epi, x, 100, 500, want_pi=False)
    a2, b2 = ctx.last_objective()
    assert b2 == pytest.approx(w[100:600].sum(), rel=1e-14)
    assert a2 == pytest.approx(float(np.dot(w[100:600], obj[100:600])), rel=1e-12)

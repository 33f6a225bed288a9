"""GPU parity of the batched stage-2 LP (solve_problem!, smps_routines.jl:50-62)
against the oracle (C dual simplex + HiGHS), through the C ABI."""
import numpy as np
import pytest

from tests import instances as I

pytestmark = pytest.mark.gpu

# baa99-20 (the instance of the reference driver, sd_single_cut_test.jl:10) has 210 negative stage-2
# costs: its start basis comes from the host phase-1 + primal simplex of twosd_compute_basis
CASES = [("lands", 512), ("newsvendor", 256), ("transship", 512), ("ssn", 512), ("storm", 512), ("baa99-20", 512)]


def _ctx(name):
    from sqlp_amd import twosd
    inst = I.load(name)
    ctx = twosd.SDContext(inst["sp2"], inst["sto"])
    x = I.x_ev(name)
    from sqlp_amd import smps
    ctx.compute_basis(x, smps.mean_values(inst["sto"]))
    return ctx, x


def test_lp_golden_fixture_baa99():
    """The committed HiGHS golden vectors of baa99-20 (tests/golden/make_golden.py): objectives
    to 1e-9 rel and strong duality of the GPU duals at the golden x and scenarios."""
    import os
    z = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "lp_baa99-20.npz"))
    from sqlp_amd import smps, twosd
    inst = I.load("baa99-20")
    ctx = twosd.SDContext(inst["sp2"], inst["sto"])
    ctx.compute_basis(z["x"], smps.mean_values(inst["sto"]))
    obj, _, pi, st = ctx.solve_values(z["x"], z["values"], want_pi=True)
    assert (st == 0).all()
    np.testing.assert_allclose(obj, z["obj"], rtol=1e-9, atol=1e-9)
    b = I.rhs_of("baa99-20", z["x"], z["values"])
    for s in range(len(obj)):
        assert abs(pi[s] @ b[s] - obj[s]) <= 1e-9 * (1 + abs(obj[s]))
        assert _dual_feasible(inst["osp2"], pi[s])


def _dual_feasible(sp, pi, tol=1e-7):
    # W' pi <= q (reduced costs of y >= 0), sign of pi by row sense
    scale = 1.0 + np.abs(sp.q).max()
    d = sp.q - sp.W.T @ pi
    ok = d.min() >= -tol * scale
    for i, s in enumerate(sp.senses):
        if s == 'G':
            ok &= pi[i] >= -tol * scale
        elif s == 'L':
            ok &= pi[i] <= tol * scale
    return ok


@pytest.mark.parametrize("name,N", CASES)
def test_lp_batch_matches_oracle(name, N):
    from oracle import cpu, lp_highs
    ctx, x = _ctx(name)
    vals = I.sample(name, N, seed=7)
    obj, y, pi, st = ctx.solve_values(x, vals, want_pi=True, want_y=True)
    assert (st == 0).all(), np.bincount(st)
    inst = I.load(name)
    sp = inst["osp2"]
    b = I.rhs_of(name, x, vals)
    # oracle C dual simplex from the same basis
    lp = cpu.CpuLP(sp.W, sp.q, sp.senses)
    lp.set_basis(ctx.get_basis())
    pos, rows, cols = __import__("sqlp_amd").smps.scenario_positions(inst["sp2"], inst["sto"])
    o_obj, o_pi, _, o_st, _ = lp.solve_batch(rows, sp.r - sp.T @ x, vals - sp.r[rows], nthreads=4)
    assert (o_st == 0).all()
    np.testing.assert_allclose(obj, o_obj, rtol=1e-9, atol=1e-9)
    # strong duality + dual feasibility of every GPU dual (obj = pi . b)
    for s in range(N):
        assert abs(pi[s] @ b[s] - obj[s]) <= 1e-9 * (1 + abs(obj[s]))
        assert _dual_feasible(sp, pi[s])
    # primal feasibility of y
    W = sp.W
    for s in range(0, N, max(1, N // 64)):
        r = W @ y[s] - b[s]
        for i, sn in enumerate(sp.senses):
            if sn == 'G':
                assert r[i] >= -1e-7 * (1 + abs(b[s][i]))
            elif sn == 'L':
                assert r[i] <= 1e-7 * (1 + abs(b[s][i]))
            else:
                assert abs(r[i]) <= 1e-7 * (1 + abs(b[s][i]))
        assert (y[s] >= -1e-9).all()
    # HiGHS objective on a subset (unique optimum)
    for s in range(0, N, max(1, N // 16)):
        hst, hobj, _, _ = lp_highs.solve_rhs(sp, b[s])
        assert hst == 0
        assert abs(hobj - obj[s]) <= 1e-8 * (1 + abs(hobj))
    # same pivot rules -> same vertex as the oracle on (almost) every scenario
    same = np.mean([np.allclose(pi[s], o_pi[s], rtol=1e-9, atol=1e-9) for s in range(N)])
    assert same >= 0.95, same


@pytest.mark.parametrize("name", ["storm", "ssn"])
def test_lp_basis_pool(name):
    """Warm-start basis pool: same optimal objectives as the oracle, valid duals; the pool
    holds distinct dual-feasible bases, primary basis first.  pool_build keeps a grown pool
    only when it saves pivots on its validation half: storm does (fewer pivots here too),
    for ssn the pool may stay at the primary basis."""
    from oracle import cpu
    from sqlp_amd import smps, twosd
    ctx, x = _ctx(name)
    inst = I.load(name)
    sp = inst["osp2"]
    head0 = ctx.get_basis()
    tr = twosd.sdEpigraph(ctx, 1.0, 0.0)
    twosd.add_scenarios(tr, I.sample(name, 2048, seed=11))
    N = 512
    vals = I.sample(name, N, seed=7)
    obj1, _, _, st1 = ctx.solve_values(x, vals)
    piv1 = ctx.lp_stats()[0]
    size = ctx.pool_build(tr, x, 0, 2048, 16)
    assert 1 <= size <= 16 and ctx.pool_size() == size
    if name == "storm":
        assert size > 1
    assert (ctx.pool_get(0) == head0).all()
    heads = [frozenset(ctx.pool_get(p).tolist()) for p in range(size)]
    assert len(set(heads)) == size
    assert not ctx.pool_add_basis(ctx.pool_get(size - 1))      # already present
    obj, _, pi, st = ctx.solve_values(x, vals, want_pi=True)
    piv = ctx.lp_stats()[0]
    assert (st == 0).all() and (st1 == 0).all()
    if name == "storm":
        assert piv < piv1, (piv, piv1)
    np.testing.assert_allclose(obj, obj1, rtol=1e-9, atol=1e-9)
    b = I.rhs_of(name, x, vals)
    lp = cpu.CpuLP(sp.W, sp.q, sp.senses)
    lp.set_basis(head0)
    pos, rows, cols = smps.scenario_positions(inst["sp2"], inst["sto"])
    o_obj, _, _, o_st, _ = lp.solve_batch(rows, sp.r - sp.T @ x, vals - sp.r[rows], nthreads=4)
    np.testing.assert_allclose(obj, o_obj, rtol=1e-9, atol=1e-9)
    for s in range(N):
        assert abs(pi[s] @ b[s] - obj[s]) <= 1e-9 * (1 + abs(obj[s]))
        assert _dual_feasible(sp, pi[s])
    # vertex parity: the oracle dual simplex started from the pool basis each scenario
    # picked reaches the same vertex (same pivot rules)
    picks = ctx.last_pool_picks(N)
    assert picks.min() >= 0 and picks.max() < size
    if name == "storm":
        assert len(np.unique(picks)) > 1
    o_pi = np.zeros_like(pi)
    for p in np.unique(picks):
        sel = np.nonzero(picks == p)[0]
        lp.set_basis(ctx.pool_get(p))
        o2, o_pi[sel], _, o2st, _ = lp.solve_batch(rows, sp.r - sp.T @ x, vals[sel] - sp.r[rows], nthreads=4)
        assert (o2st == 0).all()
        np.testing.assert_allclose(o2, obj[sel], rtol=1e-9, atol=1e-9)
    same = np.mean([np.allclose(pi[s], o_pi[s], rtol=1e-9, atol=1e-9) for s in range(N)])
    assert same >= 0.95, same
    # set_basis resets the pool
    ctx.set_basis(head0)
    assert ctx.pool_size() == 1


@pytest.mark.parametrize("groups", ["1", "3"])
def test_lp_queue_groups(groups, monkeypatch):
    """The XCD-grouped work queues (visiting order cut into qgroups contiguous ranges, idle
    waves stealing from the next range) solve every scenario exactly once: objectives and
    statuses equal the default 8-group run for 1 and 3 groups, with N not a multiple of
    either, with and without a pool-grouped visiting order."""
    from sqlp_amd import twosd
    ctx, x = _ctx("storm")
    N = 1237
    vals = I.sample("storm", N, seed=5)
    base, _, _, st0 = ctx.solve_values(x, vals)
    tr = twosd.sdEpigraph(ctx, 1.0, 0.0)
    twosd.add_scenarios(tr, I.sample("storm", 2048, seed=11))
    ctx.pool_build(tr, x, 0, 2048, 16)
    pooled, _, _, st1 = ctx.solve_values(x, vals)
    monkeypatch.setenv("TWOSD_QGROUPS", groups)
    for ref, st_ref in ((pooled, st1),):
        obj, _, _, st = ctx.solve_values(x, vals)
        assert (st == st_ref).all()
        np.testing.assert_array_equal(obj, ref)
    ctx.set_basis(ctx.get_basis())
    obj, _, _, st = ctx.solve_values(x, vals)
    assert (st == st0).all()
    np.testing.assert_array_equal(obj, base)


def test_pool_selection_picks_least_infeasible():
    """Flat warm-start selection (pool_select_kernel over the device-built selection stream,
    pool_selstream_kernel): every scenario's pick minimises the total primal infeasibility
    sum_i viol(x_B,i) of x_B = B_p^{-1} b_w over the pool, restated here in fp64 from the pool
    heads (the kernels work in fp32 and drop rows that stay feasible on the training box, which
    holds every test scenario of storm's DISCRETE distribution), up to fp32 rounding."""
    from sqlp_amd import twosd
    ctx, x = _ctx("storm")
    inst = I.load("storm")
    sp = inst["osp2"]
    tr = twosd.sdEpigraph(ctx, 1.0, 0.0)
    twosd.add_scenarios(tr, I.sample("storm", 2048, seed=11))
    P = ctx.pool_build(tr, x, 0, 2048, 16)
    assert P > 1
    N = 256
    vals = I.sample("storm", N, seed=9)
    _, _, _, st = ctx.solve_values(x, vals)
    assert (st == 0).all()
    picks = ctx.last_pool_picks(N)
    b = I.rhs_of("storm", x, vals)                    # N x m
    m, n = sp.W.shape
    tol = 1e-9
    keys = np.zeros((N, P))
    for p in range(P):
        head = ctx.pool_get(p)
        B = np.zeros((m, m))
        for i, j in enumerate(head):
            if j < n:
                B[:, i] = sp.W[:, j]
            else:
                B[j - n, i] = 1.0
        xb = np.linalg.solve(B, b.T).T                # N x m
        for i, j in enumerate(head):
            sense = None if j < n else sp.senses[j - n]
            v = xb[:, i]
            if sense == 'G':
                keys[:, p] += np.where(v > tol, v, 0.0)
            elif sense == 'E':
                keys[:, p] += np.where(np.abs(v) > tol, np.abs(v), 0.0)
            else:                                     # y_j >= 0 or slack of an L row >= 0
                keys[:, p] += np.where(v < -tol, -v, 0.0)
    best = keys.min(axis=1)
    got = keys[np.arange(N), picks]
    # fp32 evaluation: x_B entries carry ~1e-7 relative error of the rhs magnitude
    slack = 1e-4 * best + 1e-5 * (1.0 + np.abs(b).max(axis=1))
    assert (got <= best + slack).all(), np.max(got - best - slack)
    assert np.mean(got == best) > 0.9
    assert len(np.unique(picks)) > 1


def test_pool_selection_split_equals_one_chunk(monkeypatch):
    """Small batches split the pool (level 1) and the candidate lists (level 2) over several
    blocks per scenario tile and merge per scenario with the in-block rules (least key, then the
    lowest basis / the level-1 pick / the earlier candidate): the picks equal those of one chunk
    per tile (TWOSD_SEL_NOSPLIT), with the count-weighted key of device-drawn scenarios."""
    from sqlp_amd import smps, twosd
    inst = I.load("storm")
    x = I.x_ev("storm")
    ctx = twosd.SDContext(inst["sp2"], inst["sto"])
    ctx.compute_basis(x, smps.mean_values(inst["sto"]))
    ctx.set_distributions(inst["sto"])
    tr = twosd.sdEpigraph(ctx, 1.0, 0.0)
    twosd.add_sampled_scenarios(tr, 8192, 41)
    assert ctx.pool_refresh(tr, x, 0, 8192, 1024) > 128
    ctx.pool_build_candidates(tr, x, 0, 8192, 128, 160)
    ev = twosd.sdEpigraph(ctx, 1.0, 0.0)
    N = 4096
    twosd.add_sampled_scenarios(ev, N, 42)
    o1, _, _, st1 = twosd.solve_batch(ev, x, 0, N, want_pi=False)
    p1 = ctx.last_pool_picks(N)
    ctx.invalidate_x()
    monkeypatch.setenv("TWOSD_SEL_NOSPLIT", "1")
    o2, _, _, st2 = twosd.solve_batch(ev, x, 0, N, want_pi=False)
    p2 = ctx.last_pool_picks(N)
    assert (st1 == 0).all() and (st2 == 0).all()
    np.testing.assert_array_equal(p1, p2)
    np.testing.assert_array_equal(o1, o2)
    assert len(np.unique(p1)) > 128                   # level-2 candidates were picked too

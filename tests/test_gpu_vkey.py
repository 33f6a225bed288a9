"""solve_push by dual-vertex keys (vkey.hip) == pushing every scenario's dual.

push!(V, pi_s) for s = 0..N-1 (dual_set.jl:84-94) only appends the first scenario's dual of
each distinct vertex.  The default twosd_solve_push therefore solves the batch without
recovering pi, keys each optimal dual vertex by its tight dual constraints, and re-solves
only the first scenario of every key to push its pi.  TWOSD_PUSH_ALL=1 runs the direct path
(pi of every scenario pushed in order, device dedup with the reference rule).  Both must give
the identical ordered vertex set (bit for bit) and identical objectives."""
import numpy as np
import pytest

from tests import instances as I

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name,N,pool", [("lands", 3000, 1), ("transship", 6000, 1), ("ssn", 12000, 1),
                                         ("storm", 12000, 1), ("storm", 30000, 512)])
def test_keyed_push_equals_push_all(name, N, pool, monkeypatch):
    from sqlp_amd import smps, twosd
    inst = I.load(name)
    ctx = twosd.SDContext(inst["sp2"], inst["sto"])
    x = I.x_ev(name)
    ctx.compute_basis(x, smps.mean_values(inst["sto"]))
    if pool > 1:
        tr = twosd.sdEpigraph(ctx, 1.0, 0.0)
        twosd.add_scenarios(tr, I.sample(name, 4 * pool, seed=5))
        ctx.pool_build(tr, x, 0, 4 * pool, pool)
    epi = twosd.sdEpigraph(ctx, 1.0, 0.0)
    twosd.add_scenarios(epi, I.sample(name, N, seed=17))
    V = twosd.sdDualVertexSet(ctx)
    half = N // 2
    runs = []
    for mode in ("1", None):
        if mode:
            monkeypatch.setenv("TWOSD_PUSH_ALL", mode)
        else:
            monkeypatch.delenv("TWOSD_PUSH_ALL", raising=False)
        V.clear()
        objs, reps = [], []
        for lo, hi in ((0, half), (half, N)):          # two batches: the second meets a non-empty V
            obj, st, _ = twosd.solve_push(epi, x, lo, hi - lo)
            assert (st == 0).all()
            objs.append(obj)
            reps.append(ctx.last_push_reps())
        runs.append((np.concatenate(objs), V.matrix(), reps))
    (o_all, V_all, r_all), (o_key, V_key, r_key) = runs
    np.testing.assert_array_equal(o_all, o_key)
    assert V_all.shape == V_key.shape
    np.testing.assert_array_equal(V_all, V_key)
    assert r_all == [half, N - half]
    assert all(r <= c for r, c in zip(r_key, (half, N - half)))
    print(f"{name}: N={N} |V|={len(V_key)} representatives re-solved {r_key}")


@pytest.mark.parametrize("name,N,pool", [("ssn", 12000, 1), ("storm", 30000, 512), ("transship", 6000, 1)])
def test_push_full_mode_equals_resolve(name, N, pool, monkeypatch):
    """The two ways solve_push gets the representatives' duals -- re-solving them after the keyed
    main pass (TWOSD_PUSH_MODE=1), or recovering every dual in the main pass and gathering
    (TWOSD_PUSH_MODE=2) -- and the automatic choice push the same ordered V, bit for bit; the
    automatic choice switches to full mode after a batch whose representatives exceed a quarter."""
    from sqlp_amd import smps, twosd
    inst = I.load(name)
    ctx = twosd.SDContext(inst["sp2"], inst["sto"])
    x = I.x_ev(name)
    ctx.compute_basis(x, smps.mean_values(inst["sto"]))
    if pool > 1:
        tr = twosd.sdEpigraph(ctx, 1.0, 0.0)
        twosd.add_scenarios(tr, I.sample(name, 4 * pool, seed=5))
        ctx.pool_build(tr, x, 0, 4 * pool, pool)
    epi = twosd.sdEpigraph(ctx, 1.0, 0.0)
    twosd.add_scenarios(epi, I.sample(name, N, seed=17))
    V = twosd.sdDualVertexSet(ctx)
    third = N // 3
    runs = {}
    for mode in ("1", "2", "0"):
        monkeypatch.setenv("TWOSD_PUSH_MODE", mode)
        V.clear()
        objs, reps, modes = [], [], []
        for lo, hi in ((0, third), (third, 2 * third), (2 * third, N)):
            obj, st, _ = twosd.solve_push(epi, x, lo, hi - lo)
            assert (st == 0).all()
            objs.append(obj)
            reps.append(ctx.last_push_reps())
            modes.append(ctx.last_push_mode())
        runs[mode] = (np.concatenate(objs), V.matrix(), reps, modes)
    o1, V1, r1, m1 = runs["1"]
    for mode in ("2", "0"):
        o, Vm, r, _ = runs[mode]
        np.testing.assert_array_equal(o, o1)
        assert Vm.shape == V1.shape
        np.testing.assert_array_equal(Vm, V1)
        assert r == r1
    assert m1 == [0, 0, 0] and runs["2"][3] == [1, 1, 1]
    # automatic: full mode when the context's previous keyed push re-solved > 1/4 of its batch (the
    # auto run follows the mode-2 run's last batch)
    sizes = (third, third, N - 2 * third)
    frac = [r_ / n_ for r_, n_ in zip(r1, sizes)]
    assert runs["0"][3] == [int(frac[2] > 0.25), int(frac[0] > 0.25), int(frac[1] > 0.25)]
    print(f"{name}: representatives {r1}, auto modes {runs['0'][3]}")


def test_keyed_push_nonoptimal_refused():
    """A batch with a non-optimal scenario pushes nothing on the keyed path (as on the direct
    one): TWOSD_E_LP, V unchanged."""
    from sqlp_amd import smps, twosd
    from sqlp_amd._lib import TwoSDError
    inst = I.load("lands")
    ctx = twosd.SDContext(inst["sp2"], inst["sto"])
    x = I.x_ev("lands")
    ctx.compute_basis(x, smps.mean_values(inst["sto"]))
    epi = twosd.sdEpigraph(ctx, 1.0, 0.0)
    twosd.add_scenarios(epi, np.array([[5.0], [3.0], [1000.0], [7.0]]))
    V = twosd.sdDualVertexSet(ctx)
    with pytest.raises(TwoSDError):
        twosd.solve_push(epi, x, 0, 4)
    assert len(V) == 0
    twosd.solve_push(epi, x, 0, 2)
    assert len(V) >= 1 and ctx.last_push_reps() <= 2


def _sd_candidate(name, iters, seed=11):
    """x_candidate after `iters` sd_iteration! steps (host master + GPU hot path) from x_EV: a
    first-stage point of the kind the bench times, away from where any pool was trained."""
    from sqlp_amd import master, smps, twosd
    inst = I.load(name)
    sp1 = smps.get_smps_stage_template(inst["cor"], inst["tim"], 1)
    ctx = twosd.SDContext(inst["sp2"], inst["sto"])
    x0 = I.x_ev(name)
    ctx.compute_basis(x0, smps.mean_values(inst["sto"]))
    cell = master.sdCell(sp1, ctx)
    cell.bind_epigraph(twosd.sdEpigraph(ctx, 1.0, 0.0))
    cell.x_candidate = x0.copy()
    cell.x_incumbent = x0.copy()
    for it in range(iters):
        master.sd_iteration(cell, [I.sample(name, 1, seed + it)[0]])
    x = cell.x_candidate.copy()
    ctx.close()
    return x


def test_keyed_push_equals_push_all_at_scale(monkeypatch):
    """The keyed push at bench scale: storm, 262,144 scenarios, at an SD candidate (not x_EV),
    from a 4096-basis pool refreshed at that x (as every timed bench step): the ordered vertex
    set is bit-identical to pushing every scenario's pi (dual_set.jl:84-94)."""
    from sqlp_amd import smps, twosd
    inst = I.load("storm")
    x = _sd_candidate("storm", 4)
    assert np.linalg.norm(x - I.x_ev("storm")) > 1e-3 * np.linalg.norm(I.x_ev("storm"))
    ctx = twosd.SDContext(inst["sp2"], inst["sto"])
    ctx.compute_basis(I.x_ev("storm"), smps.mean_values(inst["sto"]))
    ctx.set_distributions(inst["sto"])
    tr = twosd.sdEpigraph(ctx, 1.0, 0.0)
    twosd.add_sampled_scenarios(tr, 16384, 4242)
    ctx.pool_refresh(tr, x, 0, 16384, 4096)
    assert ctx.pool_size() > 1000
    N = 262144
    epi = twosd.sdEpigraph(ctx, 1.0, 0.0)
    twosd.add_sampled_scenarios(epi, N, 777)
    V = twosd.sdDualVertexSet(ctx)
    runs = []
    for mode in (None, "1"):
        if mode:
            monkeypatch.setenv("TWOSD_PUSH_ALL", mode)
        else:
            monkeypatch.delenv("TWOSD_PUSH_ALL", raising=False)
        V.clear()
        obj, st, ns = twosd.solve_push(epi, x, 0, N)
        assert (st == 0).all()
        runs.append((obj, len(V), V.fingerprint(), ctx.last_push_reps()))
    (o_key, n_key, f_key, r_key), (o_all, n_all, f_all, r_all) = runs
    np.testing.assert_array_equal(o_key, o_all)
    assert r_all == N and r_key < N // 4
    assert (n_key, f_key) == (n_all, f_all), (n_key, n_all)
    print(f"storm {N} at SD candidate 4: |V| = {n_key}, representatives re-solved {r_key}")


def test_keyed_push_equals_reference_push_at_100k():
    """The keyed push against the reference rule itself, not the GPU's own push-all: storm, 131,072
    scenarios at x_EV from a refreshed 4096-basis pool.  Every scenario's pi (the same solves, pi
    recovered) is pushed in scenario order by the oracle's push! restatement (dual_set.jl:84-94,
    twosd_ref.DualVertexSet.push_batch); the device's keyed solve_push must build the identical
    ordered vertex set, bit for bit."""
    from oracle import twosd_ref
    from sqlp_amd import smps, twosd
    inst = I.load("storm")
    x = I.x_ev("storm")
    ctx = twosd.SDContext(inst["sp2"], inst["sto"])
    ctx.compute_basis(x, smps.mean_values(inst["sto"]))
    ctx.set_distributions(inst["sto"])
    tr = twosd.sdEpigraph(ctx, 1.0, 0.0)
    twosd.add_sampled_scenarios(tr, 16384, 4243)
    ctx.pool_refresh(tr, x, 0, 16384, 4096)
    N = 131072
    epi = twosd.sdEpigraph(ctx, 1.0, 0.0)
    twosd.add_sampled_scenarios(epi, N, 778)
    V = twosd.sdDualVertexSet(ctx)
    obj, st, _ = twosd.solve_push(epi, x, 0, N)
    assert (st == 0).all()
    reps = ctx.last_push_reps()
    Vkey = V.matrix()
    ref = twosd_ref.DualVertexSet()
    for lo in range(0, N, 16384):                      # pi of every scenario, in order
        o2, _, pis, st2 = twosd.solve_batch(epi, x, lo, 16384, want_pi=True)
        assert (st2 == 0).all()
        np.testing.assert_array_equal(o2, obj[lo:lo + 16384])
        ref.push_batch(pis)
    assert reps < N // 8
    assert Vkey.shape == ref.matrix().shape, (Vkey.shape, len(ref))
    np.testing.assert_array_equal(Vkey, ref.matrix())
    print(f"storm {N} at x_EV: |V| = {len(ref)}, representatives re-solved {reps}")

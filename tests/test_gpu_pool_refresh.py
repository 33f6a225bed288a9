"""twosd_pool_refresh: the warm-start pool rebuilt at a new first-stage point from the optimal
bases of training scenarios there, with B^{-1} composed from the eta files of their solves.
The pool only changes where each scenario starts: objectives must equal those from the
primary basis (the LP optimum is unique), every scenario stays optimal, and pivots drop."""
import numpy as np
import pytest

from tests import instances as I

pytestmark = pytest.mark.gpu


def _sd_x(n_iter=3):
    from sqlp_amd import master, smps, twosd
    inst = I.load("storm")
    sp1 = smps.get_smps_stage_template(inst["cor"], inst["tim"], 1)
    c2 = twosd.SDContext(inst["sp2"], inst["sto"])
    x0 = I.x_ev("storm")
    c2.compute_basis(x0, smps.mean_values(inst["sto"]))
    cell = master.sdCell(sp1, c2)
    cell.bind_epigraph(twosd.sdEpigraph(c2, 1.0, 0.0))
    cell.x_candidate = x0.copy()
    cell.x_incumbent = x0.copy()
    for it in range(n_iter):
        master.sd_iteration(cell, [I.sample("storm", 1, 70 + it)[0]])
    return cell.x_candidate.copy()


def test_pool_refresh_storm():
    from sqlp_amd import smps, twosd
    inst = I.load("storm")
    x_ev = I.x_ev("storm")
    x2 = _sd_x()
    assert np.linalg.norm(x2 - x_ev) > 1e-3 * np.linalg.norm(x_ev)
    ctx = twosd.SDContext(inst["sp2"], inst["sto"])
    ctx.compute_basis(x_ev, smps.mean_values(inst["sto"]))
    tr = twosd.sdEpigraph(ctx, 1.0, 0.0)
    twosd.add_scenarios(tr, I.sample("storm", 4096, seed=21))
    ctx.pool_build(tr, x_ev, 0, 4096, 256)
    ev = twosd.sdEpigraph(ctx, 1.0, 0.0)
    vals = I.sample("storm", 3000, seed=22)
    twosd.add_scenarios(ev, vals)
    ref = twosd.SDContext(inst["sp2"], inst["sto"])          # primary basis only
    ref.compute_basis(x_ev, smps.mean_values(inst["sto"]))
    o_ref, _, _, st_ref = ref.solve_values(x2, vals, want_pi=False)
    assert (st_ref == 0).all()
    o_old, _, _, st_old = twosd.solve_batch(ev, x2, 0, len(vals), want_pi=False)
    piv_old = ctx.lp_stats()[0]
    head0 = ctx.get_basis()
    P = ctx.pool_refresh(tr, x2, 0, 4096, 512)
    assert 1 < P <= 512
    np.testing.assert_array_equal(ctx.pool_get(0), head0)     # the primary basis stays pool[0]
    ms = ctx.last_refresh_ms()
    assert (ms >= 0).all() and ms[4] > 0
    o_new, _, _, st_new = twosd.solve_batch(ev, x2, 0, len(vals), want_pi=False)
    piv_new = ctx.lp_stats()[0]
    assert (st_new == 0).all()
    np.testing.assert_allclose(o_new, o_ref, rtol=1e-9, atol=1e-9)
    np.testing.assert_allclose(o_old, o_ref, rtol=1e-9, atol=1e-9)
    assert piv_new < piv_old
    # duals of the refreshed starts satisfy strong duality (vertex recovery through the composed B^{-1})
    o2, _, pi, st2 = twosd.solve_batch(ev, x2, 0, 256, want_pi=True)
    sp = inst["osp2"]
    b = np.tile(sp.r - sp.T @ x2, (256, 1))
    b[:, ctx.rows] += vals[:256] - sp.r[ctx.rows]
    np.testing.assert_allclose(np.einsum("ij,ij->i", pi, b), o2, rtol=1e-9, atol=1e-6)
    print(f"pivots/scenario {piv_old / len(vals):.2f} -> {piv_new / len(vals):.2f}, pool {P}, refresh ms {ms}")


def test_pool_refresh_bad_args():
    from sqlp_amd import smps, twosd
    from sqlp_amd._lib import TwoSDError
    inst = I.load("lands")
    ctx = twosd.SDContext(inst["sp2"], inst["sto"])
    x = I.x_ev("lands")
    ctx.compute_basis(x, smps.mean_values(inst["sto"]))
    tr = twosd.sdEpigraph(ctx, 1.0, 0.0)
    twosd.add_scenarios(tr, I.sample("lands", 64, seed=1))
    with pytest.raises(TwoSDError):
        ctx.pool_refresh(tr, x, 0, 65, 8)
    assert ctx.pool_refresh(tr, x, 0, 64, 8) <= 8


@pytest.mark.parametrize("chain", [1, 2])
def test_pool_refresh_device_build_equals_host(monkeypatch, chain):
    """The device pool build (pool_gpu.hip) and the host one (compose_binv + upload_pool +
    prepare_elements, TWOSD_REFRESH_HOST=1) produce the same pool: the same bases, and solves
    from it with identical objectives and pivot counts.  chain = 2 refreshes twice, so the second
    composes from device-built start bases; afterwards a host-side pool change (pool_build,
    which reads every basis back in host form) must keep the objectives exact."""
    from sqlp_amd import smps, twosd
    inst = I.load("storm")
    x_ev = I.x_ev("storm")
    x2 = _sd_x()
    x3 = x_ev + 0.6 * (x2 - x_ev)
    xs = [x2, x3][:chain]
    vals = I.sample("storm", 3000, seed=23)
    runs = []
    for mode in ("host", "device"):
        if mode == "host":
            monkeypatch.setenv("TWOSD_REFRESH_HOST", "1")
        else:
            monkeypatch.delenv("TWOSD_REFRESH_HOST", raising=False)
        ctx = twosd.SDContext(inst["sp2"], inst["sto"])
        ctx.compute_basis(x_ev, smps.mean_values(inst["sto"]))
        tr = twosd.sdEpigraph(ctx, 1.0, 0.0)
        twosd.add_scenarios(tr, I.sample("storm", 4096, seed=21))
        ctx.pool_build(tr, x_ev, 0, 4096, 256)
        ev = twosd.sdEpigraph(ctx, 1.0, 0.0)
        twosd.add_scenarios(ev, vals)
        for x in xs:
            P = ctx.pool_refresh(tr, x, 0, 4096, 512)
        o, _, _, st = twosd.solve_batch(ev, xs[-1], 0, len(vals), want_pi=False)
        runs.append((P, [ctx.pool_get(p) for p in range(P)], o, st, ctx.lp_stats()[0], ctx, tr, ev))
    (P_h, heads_h, o_h, st_h, piv_h, _, _, _), (P_d, heads_d, o_d, st_d, piv_d, ctx, tr, ev) = runs
    assert P_h == P_d
    for a, b in zip(heads_h, heads_d):
        np.testing.assert_array_equal(a, b)
    assert (st_h == 0).all() and (st_d == 0).all()
    np.testing.assert_allclose(o_d, o_h, rtol=1e-12, atol=1e-12)
    assert piv_d == piv_h
    ref = twosd.SDContext(inst["sp2"], inst["sto"])
    ref.compute_basis(x_ev, smps.mean_values(inst["sto"]))
    o_ref, _, _, _ = ref.solve_values(xs[-1], vals, want_pi=False)
    ctx.pool_build(tr, x_ev, 0, 4096, P_d + 64)          # host path over the device-built pool
    o_after, _, _, st_after = twosd.solve_batch(ev, xs[-1], 0, len(vals), want_pi=False)
    assert (st_after == 0).all()
    np.testing.assert_allclose(o_after, o_ref, rtol=1e-9, atol=1e-9)
    print(f"chain {chain}: pool {P_d}, pivots {piv_d / len(vals):.2f}, refresh ms {ctx.last_refresh_ms()}")


@pytest.mark.parametrize("name,N,train,pool", [("ssn", 4000, 2048, 256), ("lands", 2000, 512, 32),
                                               ("transship", 2000, 1024, 64)])
def test_pool_refresh_device_build_other_instances(monkeypatch, name, N, train, pool):
    """Device vs host pool build on the other instances (different m, k, element rows per
    column, fixed basics): same pool, same objectives and pivots; objectives equal the
    primary-basis solve."""
    from sqlp_amd import smps, twosd
    inst = I.load(name)
    x_ev = I.x_ev(name)
    x2 = x_ev * 1.07 + 0.01
    vals = I.sample(name, N, seed=31)
    runs = []
    for mode in ("host", "device"):
        if mode == "host":
            monkeypatch.setenv("TWOSD_REFRESH_HOST", "1")
        else:
            monkeypatch.delenv("TWOSD_REFRESH_HOST", raising=False)
        ctx = twosd.SDContext(inst["sp2"], inst["sto"])
        ctx.compute_basis(x_ev, smps.mean_values(inst["sto"]))
        tr = twosd.sdEpigraph(ctx, 1.0, 0.0)
        twosd.add_scenarios(tr, I.sample(name, train, seed=32))
        ctx.pool_build(tr, x_ev, 0, train, pool)
        ev = twosd.sdEpigraph(ctx, 1.0, 0.0)
        twosd.add_scenarios(ev, vals)
        P = ctx.pool_refresh(tr, x2, 0, train, pool)
        o, _, _, st = twosd.solve_batch(ev, x2, 0, N, want_pi=False)
        runs.append((P, [ctx.pool_get(p) for p in range(P)], o, st, ctx.lp_stats()[0]))
    (P_h, heads_h, o_h, st_h, piv_h), (P_d, heads_d, o_d, st_d, piv_d) = runs
    assert P_h == P_d and P_d >= 1
    for a, b in zip(heads_h, heads_d):
        np.testing.assert_array_equal(a, b)
    np.testing.assert_array_equal(st_h, st_d)
    np.testing.assert_allclose(o_d, o_h, rtol=1e-12, atol=1e-12)
    assert piv_d == piv_h
    ref = twosd.SDContext(inst["sp2"], inst["sto"])
    ref.compute_basis(x_ev, smps.mean_values(inst["sto"]))
    o_ref, _, _, st_ref = ref.solve_values(x2, vals, want_pi=False)
    ok = (st_ref == 0) & (st_d == 0)
    assert ok.mean() > 0.95
    np.testing.assert_allclose(o_d[ok], o_ref[ok], rtol=1e-9, atol=1e-7)
    print(f"{name}: pool {P_d}, pivots {piv_d / N:.2f}")


def test_refresh_failure_leaves_context_refusing(monkeypatch):
    """A device pool build that fails after the live pool arrays were grown (injected here,
    TWOSD_INJECT_FAIL=refresh_fill) leaves no pool pointing at stale arrays: the refresh raises,
    every later solve is refused (TWOSD_E_STATE) until a basis is installed again, and then the
    context solves as before."""
    from sqlp_amd import smps, twosd
    from sqlp_amd._lib import TwoSDError
    inst = I.load("storm")
    x = I.x_ev("storm")
    ctx = twosd.SDContext(inst["sp2"], inst["sto"])
    mean = smps.mean_values(inst["sto"])
    ctx.compute_basis(x, mean)
    vals = I.sample("storm", 256, seed=3)
    ref, _, _, st = ctx.solve_values(x, vals)
    assert (st == 0).all()
    tr = twosd.sdEpigraph(ctx, 1.0, 0.0)
    twosd.add_scenarios(tr, I.sample("storm", 2048, seed=11))
    monkeypatch.setenv("TWOSD_INJECT_FAIL", "refresh_fill")
    with pytest.raises(TwoSDError) as e:
        ctx.pool_refresh(tr, x, 0, 2048, 512)
    assert e.value.code == -2
    monkeypatch.delenv("TWOSD_INJECT_FAIL")
    with pytest.raises(TwoSDError) as e:
        ctx.solve_values(x, vals)
    assert e.value.code == -3
    ctx.compute_basis(x, mean)
    obj, _, _, st = ctx.solve_values(x, vals)
    assert (st == 0).all()
    np.testing.assert_array_equal(obj, ref)
    assert ctx.pool_refresh(tr, x, 0, 2048, 512) > 1        # and refreshes again
    obj, _, _, st = ctx.solve_values(x, vals)
    np.testing.assert_allclose(obj, ref, rtol=1e-9, atol=1e-9)


def test_refresh_training_cap_too_low_is_solved_again():
    """A training cap far below the pivots the jump to a new x needs (bench with warmup 4: the
    x_EV pool, next x an SD candidate, cap 35 against 58.5 pivots a scenario) used to leave the
    refresh with no optimal training scenario and the pool at the primary basis alone.  With
    fewer than half of the training solves optimal, the refresh solves them again uncapped."""
    from sqlp_amd import smps, twosd
    inst = I.load("storm")
    x_ev = I.x_ev("storm")
    x2 = _sd_x()
    ctx = twosd.SDContext(inst["sp2"], inst["sto"])
    ctx.compute_basis(x_ev, smps.mean_values(inst["sto"]))
    tr = twosd.sdEpigraph(ctx, 1.0, 0.0)
    twosd.add_scenarios(tr, I.sample("storm", 4096, seed=31))
    assert ctx.pool_refresh(tr, x_ev, 0, 4096, 512) > 1
    ev = twosd.sdEpigraph(ctx, 1.0, 0.0)
    vals = I.sample("storm", 2000, seed=32)
    twosd.add_scenarios(ev, vals)
    ctx.set_refresh_kcap(3)                     # almost no training scenario reaches optimality
    P = ctx.pool_refresh(tr, x2, 0, 4096, 512)
    assert P > 256                              # rebuilt from the uncapped training solves
    o, _, _, st = twosd.solve_batch(ev, x2, 0, len(vals), want_pi=False)
    assert (st == 0).all()
    assert ctx.lp_stats()[0] / len(vals) < 20   # a pool at x2, not the primary basis alone
    ctx.set_refresh_kcap(0)


@pytest.mark.parametrize("mode", ["scratch_small", "two_pass"])
def test_pool_build_single_ftran_pass_identical(monkeypatch, capfd, mode):
    """The pool build keeps the first FTRAN pass's nonzeros and gathers the kept entries from
    them (pg_gather_kernel); sources past the scratch take the second FTRAN pass.  Against the
    two-pass build (TWOSD_PG_NOSCRATCH) and a scratch so small that only some sources fit
    (TWOSD_PG_SCCAP), the refreshed pool solves the same scenarios with bit-identical objectives
    and the same pivots."""
    from sqlp_amd import smps, twosd
    inst = I.load("storm")
    x_ev = I.x_ev("storm")
    x2 = _sd_x()
    vals = I.sample("storm", 3000, seed=41)
    runs = []
    cap_mid = None
    for variant in ("default", mode):
        monkeypatch.delenv("TWOSD_PG_NOSCRATCH", raising=False)
        monkeypatch.delenv("TWOSD_PG_SCCAP", raising=False)
        monkeypatch.setenv("TWOSD_DEBUG", "1")
        if variant == "two_pass":
            monkeypatch.setenv("TWOSD_PG_NOSCRATCH", "1")
        elif variant == "scratch_small":     # the mean source: about half of them take pass 1
            monkeypatch.setenv("TWOSD_PG_SCCAP", str(cap_mid))
        ctx = twosd.SDContext(inst["sp2"], inst["sto"])
        ctx.compute_basis(x_ev, smps.mean_values(inst["sto"]))
        tr = twosd.sdEpigraph(ctx, 1.0, 0.0)
        twosd.add_scenarios(tr, I.sample("storm", 4096, seed=42))
        ctx.pool_build(tr, x_ev, 0, 4096, 256)
        ev = twosd.sdEpigraph(ctx, 1.0, 0.0)
        twosd.add_scenarios(ev, vals)
        P = ctx.pool_refresh(tr, x2, 0, 4096, 512)
        P = ctx.pool_refresh(tr, x_ev, 0, 4096, 512)      # the second refresh composes from device-built bases
        o, _, _, st = twosd.solve_batch(ev, x_ev, 0, len(vals), want_pi=False)
        it, _ = ctx.last_lp_iters(len(vals))
        runs.append((P, [ctx.pool_get(p) for p in range(P)], o, st, it))
        builds = [ln.split() for ln in capfd.readouterr().err.splitlines() if ln.startswith("pg_compute:")]
        assert len(builds) >= 2
        # "pg_compute: S sources, Z intermediate entries, largest L, O past the scratch of C"
        S, Z, O = int(builds[-1][1]), int(builds[-1][3]), int(builds[-1][8])
        if variant == "default":
            assert O == 0                    # the scratch (sized by the first build) held every source
            cap_mid = Z // S
        elif variant == "scratch_small":
            assert 0 < O < S                 # some sources, not all, took the second FTRAN pass
    (P_a, h_a, o_a, st_a, it_a), (P_b, h_b, o_b, st_b, it_b) = runs
    assert P_a == P_b and P_a > 64
    for a, b in zip(h_a, h_b):
        np.testing.assert_array_equal(a, b)
    np.testing.assert_array_equal(st_a, st_b)
    np.testing.assert_array_equal(o_a, o_b)
    np.testing.assert_array_equal(it_a, it_b)

"""Config C3 (ssn, large dual-vertex set, MFMA argmax stressed) under parity: V grown to
16,384 and then 65,536 real LP duals (twosd_solve_push over ssn scenarios, so the cut's
vertex staging is rebuilt as the set grows), then argmax_procedure + build_sasa_cut
(subprob.jl:141-169, epigraph.jl:125-146) over 2,000 weighted scenarios on the GPU against
the reference-order C port (oracle/cpu_lp.c): the same argmax for every scenario (near ties
included), alpha / beta within 1e-8 relative (north star), the global-atomic vertex histogram path
(|V| > 256) included."""
import numpy as np
import pytest

from tests import instances as I

pytestmark = pytest.mark.gpu


def _grow(ctx, epi, x, target, state):
    from sqlp_amd import twosd
    V = twosd.sdDualVertexSet(ctx)
    while len(V) < target:
        first = state["next"]
        if first + 16384 > epi.num_scenarios:
            raise AssertionError(f"only {len(V)} distinct duals from {first} scenarios")
        _, st, _ = twosd.solve_push(epi, x, first, 16384)
        assert (st == 0).all()
        state["next"] = first + 16384
    V.truncate(target)
    return V


def _check(ctx, x, V, vals, w, tie_rel):
    from oracle import cpu
    from sqlp_amd import twosd
    sp = I.load("ssn")["osp2"]
    epi = twosd.sdEpigraph(ctx, 1.0, 0.0)
    twosd.add_scenarios(epi, vals, w)
    cut, mv, ma = twosd._build_cut(epi, x, tie_rel, want_argmax=True)
    Vm = V.matrix()
    a, b, omv, oma = cpu.build_cut(sp.r, sp.T, x, Vm, ctx.rows, vals - sp.r[ctx.rows], w, tie_rel=tie_rel, nthreads=8)
    N = vals.shape[0]
    np.testing.assert_allclose(mv, omv, rtol=1e-10, atol=1e-9)
    scores = (Vm @ (sp.r - sp.T @ x))[None, :] + (vals - sp.r[ctx.rows]) @ Vm[:, ctx.rows].T
    part = np.partition(scores, -2, axis=1)[:, -2:]
    top, second = part.max(1), part.min(1)
    clear = (top - second) > 1e-9 * (1 + np.abs(top))
    assert clear.mean() > 0.5
    assert (ma == oma).all(), (tie_rel, int((~clear).sum()), int((ma != oma).sum()))   # near ties included
    assert (scores[np.arange(N), ma] >= top - 1e-9 * (1 + np.abs(top))).all()
    assert cut.alpha == pytest.approx(a, rel=1e-8)
    np.testing.assert_allclose(cut.beta, b, rtol=1e-8, atol=1e-8 * (1 + np.abs(b).max()))
    p = w / w.sum()
    ra = np.tile(sp.r, (N, 1))
    ra[:, ctx.rows] = vals
    a_ref = float(np.sum(p * np.einsum("ij,ij->i", Vm[ma], ra)))
    b_ref = -(sp.T.T @ (p @ Vm[ma]))
    assert cut.alpha == pytest.approx(a_ref, rel=1e-9)
    np.testing.assert_allclose(cut.beta, b_ref, rtol=1e-9, atol=1e-9 * (1 + np.abs(b_ref).max()))
    return ma


def test_large_vertex_set_cut_ssn():
    from sqlp_amd import smps, twosd
    inst = I.load("ssn")
    ctx = twosd.SDContext(inst["sp2"], inst["sto"])
    x = I.x_ev("ssn")
    ctx.compute_basis(x, smps.mean_values(inst["sto"]))
    src = twosd.sdEpigraph(ctx, 1.0, 0.0)
    ctx.set_distributions(inst["sto"])
    twosd.add_sampled_scenarios(src, 16384 * 8, seed=2024)
    state = {"next": 0}
    vals = I.sample("ssn", 2000, seed=99)
    w = np.random.default_rng(6).uniform(0.5, 1.5, size=2000)
    V = _grow(ctx, src, x, 16384, state)
    assert len(V) == 16384
    _check(ctx, x, V, vals, w, 1e-12)
    V = _grow(ctx, src, x, 65536, state)                # the cut's vertex staging grows
    assert len(V) == 65536
    ma = _check(ctx, x, V, vals, w, 1e-12)
    assert ma.max() >= 16384                            # picks among the added vertices
    _check(ctx, x, V, vals, w, 0.0)


@pytest.mark.parametrize("name,N,nsrc", [("ssn", 100_000, 12000), ("storm", 70_000, 16384)])
def test_tail_split_equals_whole_tiles(name, N, nsrc, monkeypatch):
    """The last round of the cut's persistent grid cut into vertex ranges (cut_tail_merge_kernel)
    decides every scenario as the whole-tile pass does: identical argmax, max_val, alpha/beta
    (TWOSD_CUT_TAIL=0 turns the split off)."""
    from sqlp_amd import smps, twosd
    inst = I.load(name)
    ctx = twosd.SDContext(inst["sp2"], inst["sto"])
    x = I.x_ev(name)
    ctx.compute_basis(x, smps.mean_values(inst["sto"]))
    V = twosd.sdDualVertexSet(ctx)
    _, _, pis, st = ctx.solve_values(x, I.sample(name, nsrc, 3), want_pi=True)
    V.push_batch(pis[st == 0])
    assert len(V) >= 512
    epi = twosd.sdEpigraph(ctx, 1.0, 0.0)
    twosd.add_scenarios(epi, I.sample(name, N, 17), np.random.default_rng(2).uniform(0.5, 1.5, N))
    res = []
    for tail in ("1", "0"):
        monkeypatch.setenv("TWOSD_CUT_TAIL", tail)
        res.append(twosd._build_cut(epi, x, 1e-12, want_argmax=True))
    (c1, mv1, ma1), (c0, mv0, ma0) = res
    np.testing.assert_array_equal(ma1, ma0)
    np.testing.assert_array_equal(mv1, mv0)
    assert c1.alpha == pytest.approx(c0.alpha, rel=1e-13, abs=1e-13)
    np.testing.assert_allclose(c1.beta, c0.beta, rtol=1e-13, atol=1e-13)

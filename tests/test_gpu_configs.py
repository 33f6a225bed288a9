"""BASELINE configs at their real per-rank size against the oracle.

* C4 -- storm, 1M scenarios sharded over 8 GPUs: one rank's 125,000-scenario shard (rank 3 of the
  device-drawn stream, so the shard starts at scenario 375,000) with |V| = 4,096 real duals built at
  x_EV as the bench builds them.  Every LP objective against the C dual simplex, and the cut at
  x_EV (where V was built: twin-rich, many exact ties) under the reference's strict '>' and the
  near-tie rule: max_arg equal for EVERY scenario, alpha / beta to 1e-8 (epigraph.jl:125-146).
* C5 -- transship, 4 weighted epigraphs x 250,000 importance-sampled scenarios on one GPU (the
  bench's --epigraphs 4 --importance-scale 1.5 stream and weights): each epigraph's cut against
  cpu.build_cut, max_arg exact, alpha / beta to 1e-8.
The RCCL leg of both configs needs an 8-GPU node and is not exercised here."""
import os

import numpy as np
import pytest

from tests import instances as I

pytestmark = pytest.mark.gpu


def _threads():
    return max(1, min(16, len(os.sched_getaffinity(0))))


def _storm_V(ctx, x, nv, seed):
    """The bench's |V| pool: distinct duals of the stream `seed` solved at x, in order, cut at nv."""
    from sqlp_amd import twosd
    V = twosd.sdDualVertexSet(ctx)
    src = twosd.sdEpigraph(ctx, 1.0, 0.0)
    twosd.add_sampled_scenarios(src, 1 << 17, seed)
    at = 0
    while len(V) < nv and at < (1 << 17):
        _, _, pis, st = twosd.solve_batch(src, x, at, 16384, want_pi=True)
        V.push_batch(pis[st == 0])
        at += 16384
    if len(V) > nv:
        V.truncate(nv)
    return V


def test_c4_storm_125k_shard_at_4096_vertices():
    from oracle import cpu
    from sqlp_amd import smps, twosd
    inst = I.load("storm")
    sp2, sto = inst["sp2"], inst["sto"]
    x = I.x_ev("storm")
    ctx = twosd.SDContext(sp2, sto)
    ctx.compute_basis(x, smps.mean_values(sto))
    ctx.set_distributions(sto)
    V = _storm_V(ctx, x, 4096, seed=20250220)
    assert len(V) == 4096
    N = 125_000
    epi = twosd.sdEpigraph(ctx, 1.0, 0.0)
    twosd.add_sampled_scenarios(epi, N, 20250219, first_index=3 * N)
    # a refreshed pool at x (the bench's per-x protocol), then every LP of the shard
    tr = twosd.sdEpigraph(ctx, 1.0, 0.0)
    twosd.add_sampled_scenarios(tr, 4096, 20250223)
    ctx.pool_refresh(tr, x, 0, 4096, 512)
    ctx.pool_build_candidates(tr, x, 0, 4096, 128, 160)
    obj, _, _, st = twosd.solve_batch(epi, x, 0, N, want_pi=False)
    assert (st == 0).all()
    vals = twosd.get_scenarios(epi, 0, N)
    sp = inst["osp2"]
    rows = ctx.rows
    DR = vals - sp.r[rows]
    lp = cpu.CpuLP(sp2.dense_W(), sp2.q, sp2.sense)
    lp.set_basis(ctx.get_basis())
    o_obj, _, _, o_st, _ = lp.solve_batch(rows, sp.r - sp.T @ x, DR, nthreads=_threads())
    assert (o_st == 0).all()
    np.testing.assert_allclose(obj, o_obj, rtol=1e-9, atol=1e-9)
    Vm = V.matrix()
    for tie_rel in (0.0, 1e-12):
        cut, mv, ma = twosd._build_cut(epi, x, tie_rel, want_argmax=True)
        a, b, omv, oma = cpu.build_cut(sp.r, sp.T, x, Vm, rows, DR, np.ones(N), tie_rel=tie_rel, nthreads=_threads())
        assert (ma == oma).all(), (tie_rel, int((ma != oma).sum()))
        np.testing.assert_allclose(mv, omv, rtol=1e-12, atol=1e-9)
        assert cut.alpha == pytest.approx(a, rel=1e-8, abs=1e-8)
        np.testing.assert_allclose(cut.beta, b, rtol=1e-8, atol=1e-8 * (1 + np.abs(b).max()))
        if tie_rel == 0.0:
            assert ctx.cut_stats()[3] > 0            # dominated twins of V left out of the MFMA pass


def test_c5_transship_4x250k_importance_weighted():
    import bench
    from oracle import cpu
    from sqlp_amd import smps, twosd
    inst = I.load("transship")
    sp2, sto = inst["sp2"], inst["sto"]
    x = I.x_ev("transship")
    ctx = twosd.SDContext(sp2, sto)
    ctx.compute_basis(x, smps.mean_values(sto))
    V = twosd.sdDualVertexSet(ctx)
    _, _, pis, st = ctx.solve_values(x, I.sample("transship", 4096, 3), want_pi=True)
    V.push_batch(pis[st == 0])
    Vm = V.matrix()
    sp = inst["osp2"]
    positions = list(sto.indep.keys())
    E, NE = 4, 250_000
    seed = 20250219
    for e in range(E):
        vals, w = bench.importance_values(sto, positions, 0, NE, seed + 101 * (e + 1), 1.5)
        epi = twosd.sdEpigraph(ctx, 1.0 / E, 0.0)
        twosd.add_scenarios(epi, vals, w)
        assert epi.total_scenario_weight == pytest.approx(w.sum(), rel=1e-13)
        cut, mv, ma = twosd._build_cut(epi, x, 0.0, want_argmax=True)
        a, b, omv, oma = cpu.build_cut(sp.r, sp.T, x, Vm, ctx.rows, vals - sp.r[ctx.rows], w, tie_rel=0.0,
                                       nthreads=_threads())
        assert (ma == oma).all(), (e, int((ma != oma).sum()))
        np.testing.assert_allclose(mv, omv, rtol=1e-12, atol=1e-9)
        assert cut.alpha == pytest.approx(a, rel=1e-8, abs=1e-8)
        np.testing.assert_allclose(cut.beta, b, rtol=1e-8, atol=1e-8 * (1 + np.abs(b).max()))
        assert cut.weight_mark == pytest.approx(w.sum(), rel=1e-13)

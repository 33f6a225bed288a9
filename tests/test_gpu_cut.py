"""GPU argmax_procedure + build_sasa_cut (subprob.jl:141-169, epigraph.jl:125-146) vs the
oracle: reference-order C port on the same V / scenarios / weights, the golden fixtures,
multi-epigraph importance weights (config C5) and the sharded partial/finalize API."""
import os

import numpy as np
import pytest

from tests import instances as I

pytestmark = pytest.mark.gpu
G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


class _env:
    """Set one environment variable for a block (the library reads TWOSD_CUT_TWINS per cut)."""

    def __init__(self, key, value):
        self.key, self.value = key, value

    def __enter__(self):
        self.old = os.environ.get(self.key)
        os.environ[self.key] = self.value

    def __exit__(self, *a):
        if self.old is None:
            os.environ.pop(self.key, None)
        else:
            os.environ[self.key] = self.old


def _setup(name, nv_src=512, seed=3):
    from sqlp_amd import smps, twosd
    inst = I.load(name)
    ctx = twosd.SDContext(inst["sp2"], inst["sto"])
    x = I.x_ev(name)
    ctx.compute_basis(x, smps.mean_values(inst["sto"]))
    V = twosd.sdDualVertexSet(ctx)
    _, _, pis, st = ctx.solve_values(x, I.sample(name, nv_src, seed), want_pi=True)
    V.push_batch(pis[st == 0])
    return ctx, x, V


@pytest.mark.parametrize("name,N", [("lands", 300), ("newsvendor", 200), ("transship", 700), ("ssn", 1500),
                                    ("storm", 1000), ("baa99-20", 800)])
@pytest.mark.parametrize("tie_rel", [0.0, 1e-12])
def test_cut_matches_oracle(name, N, tie_rel):
    from oracle import cpu
    from sqlp_amd import twosd
    ctx, x, V = _setup(name)
    vals = I.sample(name, N, seed=17)
    w = np.random.default_rng(5).uniform(0.5, 1.5, size=N)
    epi = twosd.sdEpigraph(ctx, 1.0, 0.0)
    twosd.add_scenarios(epi, vals, w)
    cut, mv, ma = twosd._build_cut(epi, x, tie_rel, want_argmax=True)
    sp = I.load(name)["osp2"]
    Vm = V.matrix()
    a, b, omv, oma = cpu.build_cut(sp.r, sp.T, x, Vm, ctx.rows, vals - sp.r[ctx.rows], w, tie_rel=tie_rel, nthreads=4)
    assert cut.weight_mark == pytest.approx(w.sum(), rel=1e-15)
    np.testing.assert_allclose(mv, omv, rtol=1e-10, atol=1e-9)
    scores = (Vm @ (sp.r - sp.T @ x))[None, :] + (vals - sp.r[ctx.rows]) @ Vm[:, ctx.rows].T
    top2 = np.sort(scores, axis=1)[:, -2:] if Vm.shape[0] > 1 else np.hstack([scores, scores - 1])
    ties = int(((top2[:, 1] - top2[:, 0]) <= 1e-9 * (1 + np.abs(top2[:, 1]))).sum())
    # argmax: the oracle's pick for every scenario, near ties included (the GPU re-decides them
    # in the restatement's arithmetic)
    assert (ma == oma).all(), (ties, int((ma != oma).sum()))
    best = scores.max(1)
    assert (scores[np.arange(N), ma] >= best - 1e-9 * (1 + np.abs(best))).all()
    assert cut.alpha == pytest.approx(a, rel=1e-8, abs=1e-8)        # north star: 1e-8 rel
    np.testing.assert_allclose(cut.beta, b, rtol=1e-8, atol=1e-8 * (1 + np.abs(b).max()))
    # the cut equals the reference formula (epigraph.jl:134-143) over the GPU's own choices
    p = w / w.sum()
    ra = np.tile(sp.r, (N, 1))
    ra[:, ctx.rows] = vals
    a_ref = float(np.sum(p * np.einsum("ij,ij->i", Vm[ma], ra)))
    b_ref = -(sp.T.T @ (p @ Vm[ma]))
    assert cut.alpha == pytest.approx(a_ref, rel=1e-9, abs=1e-9)
    np.testing.assert_allclose(cut.beta, b_ref, rtol=1e-9, atol=1e-9 * (1 + np.abs(b_ref).max()))


@pytest.mark.parametrize("name", ["lands", "newsvendor", "transship", "ssn", "storm", "baa99-20"])
def test_cut_golden_fixture(name):
    from sqlp_amd import twosd
    z = np.load(os.path.join(G, f"cut_{name}.npz"))
    inst = I.load(name)
    ctx = twosd.SDContext(inst["sp2"], inst["sto"])
    V = twosd.sdDualVertexSet(ctx)
    idx = V.push_batch(z["V"])
    assert idx.tolist() == list(range(len(z["V"])))
    epi = twosd.sdEpigraph(ctx, 1.0, 0.0)
    twosd.add_scenarios(epi, z["values"], z["w"])
    cut, mv, ma = twosd._build_cut(epi, z["x"], 0.0, want_argmax=True)
    assert (ma == z["max_arg"]).all()
    assert cut.alpha == pytest.approx(float(z["alpha"]), rel=1e-8)
    np.testing.assert_allclose(cut.beta, z["beta"], rtol=1e-8, atol=1e-8)
    np.testing.assert_allclose(mv, z["max_val"], rtol=1e-10, atol=1e-9)


def test_multi_epigraph_importance_weights():
    """Config C5 shape: transship, 4 epigraphs (objective weight 0.25), scenarios drawn from
    N(mu, (1.5 sigma)^2) with likelihood-ratio weights, a shared vertex set."""
    from oracle import cpu
    from sqlp_amd import twosd
    ctx, x, V = _setup("transship", 2048)
    sto = I.load("transship")["sto"]
    mu = np.array([d[1] for d in sto.indep.values()])
    sd = np.sqrt([d[2] for d in sto.indep.values()])
    rng = np.random.default_rng(8)
    sp = I.load("transship")["osp2"]
    Vm = V.matrix()
    for e in range(4):
        epi = twosd.sdEpigraph(ctx, 0.25, 0.0)
        vals = rng.normal(mu, 1.5 * sd, size=(600, len(mu)))
        logw = (-0.5 * ((vals - mu) / sd) ** 2).sum(1) - (-0.5 * ((vals - mu) / (1.5 * sd)) ** 2).sum(1) + len(mu) * np.log(1.5)
        w = np.exp(logw)
        twosd.add_scenarios(epi, vals, w)
        cut = twosd.build_sasa_cut(epi, x, V, tie_rel=1e-12)
        a, b, _, _ = cpu.build_cut(sp.r, sp.T, x, Vm, ctx.rows, vals - sp.r[ctx.rows], w, tie_rel=1e-12)
        assert cut.alpha == pytest.approx(a, rel=1e-8)
        np.testing.assert_allclose(cut.beta, b, rtol=1e-8, atol=1e-8)
        assert epi.total_scenario_weight == pytest.approx(w.sum(), rel=1e-14)


def test_sharded_partials_equal_single_cut():
    """twosd_cut_partial on two scenario shards + host sum (the all-reduce) + finalize ==
    twosd_build_cut over all scenarios; the uint64 vertex histogram is bit-identical."""
    import torch
    from sqlp_amd import twosd
    ctx, x, V = _setup("ssn", 1024)
    vals = I.sample("ssn", 2000, seed=21)
    w = np.random.default_rng(1).uniform(0.5, 1.5, size=2000)
    full = twosd.sdEpigraph(ctx, 1.0, 0.0)
    twosd.add_scenarios(full, vals, w)
    ref = twosd.build_sasa_cut(full, x, V, tie_rel=1e-12)
    halves = [twosd.sdEpigraph(ctx, 1.0, 0.0) for _ in range(2)]
    twosd.add_scenarios(halves[0], vals[:900], w[:900])
    twosd.add_scenarios(halves[1], vals[900:], w[900:])
    nu, nf = ctx.cut_partial_len()
    dev = torch.device("cuda", 0)
    H = [torch.zeros(nu, dtype=torch.int64, device=dev) for _ in range(2)]
    S = [torch.zeros(nf, dtype=torch.float64, device=dev) for _ in range(2)]
    hist1 = torch.zeros(nu, dtype=torch.int64, device=dev)
    sums1 = torch.zeros(nf, dtype=torch.float64, device=dev)
    ctx.cut_partial(full, x, 1e-12, w.sum(), hist1.data_ptr(), sums1.data_ptr())
    for e in range(2):
        ctx.cut_partial(halves[e], x, 1e-12, w.sum(), H[e].data_ptr(), S[e].data_ptr())
    torch.cuda.synchronize()
    hist = H[0] + H[1]
    sums = S[0] + S[1]
    assert torch.equal(hist, hist1)
    a, b = ctx.cut_finalize(x, hist.data_ptr(), sums.data_ptr())
    assert a == pytest.approx(ref.alpha, rel=1e-12)
    np.testing.assert_allclose(b, ref.beta, rtol=1e-12, atol=1e-12)


def test_empty_vertex_set_raises():
    from sqlp_amd import twosd
    from sqlp_amd._lib import TwoSDError
    inst = I.load("lands")
    ctx = twosd.SDContext(inst["sp2"], inst["sto"])
    epi = twosd.sdEpigraph(ctx, 1.0, 0.0)
    twosd.add_scenarios(epi, I.sample("lands", 4, 1))
    with pytest.raises(TwoSDError):            # UndefRefError in build_sasa_cut (epigraph.jl:140)
        twosd.build_sasa_cut(epi, I.x_ev("lands"), twosd.sdDualVertexSet(ctx))


def test_cut_ssn_full_rounds_three_blocks_per_cu():
    """ssn's 22 k-blocks run the cut kernel at 3 blocks per CU; at 120k scenarios (938 tiles) the
    persistent grid runs whole-tile rounds and then the vertex-split tail.  Against the C oracle
    under both tie rules: the same argmax for every scenario, alpha and beta to 1e-8."""
    from oracle import cpu
    from sqlp_amd import twosd
    ctx, x, V = _setup("ssn", nv_src=768)
    N = 120_000
    vals = I.sample("ssn", N, seed=29)
    w = np.random.default_rng(7).uniform(0.5, 1.5, size=N)
    epi = twosd.sdEpigraph(ctx, 1.0, 0.0)
    twosd.add_scenarios(epi, vals, w)
    sp = I.load("ssn")["osp2"]
    for tie_rel in (1e-12, 0.0):
        cut, mv, ma = twosd._build_cut(epi, x, tie_rel, want_argmax=True)
        a, b, omv, oma = cpu.build_cut(sp.r, sp.T, x, V.matrix(), ctx.rows, vals - sp.r[ctx.rows], w, tie_rel=tie_rel,
                                       nthreads=8)
        assert (ma == oma).all(), (tie_rel, int((ma != oma).sum()))
        np.testing.assert_allclose(mv, omv, rtol=1e-10, atol=1e-9)
        assert cut.alpha == pytest.approx(a, rel=1e-8, abs=1e-8)
        np.testing.assert_allclose(cut.beta, b, rtol=1e-8, atol=1e-8 * (1 + np.abs(b).max()))


def test_cut_storm_at_the_x_where_V_was_built():
    """The representative SD case (algorithm.jl:45-55, 79-85: the cut is built at the x whose
    duals were just pushed): storm at x_EV, V = the distinct duals of 16,384 scenarios solved
    there, the cut over 4,096 other scenarios at the same x.  Most scenarios are degenerate and
    several of their optimal vertices are in V (exact ties).  Under the reference's strict '>'
    (tie_rel = 0) and the near-tie rule: max_arg identical to the C oracle for EVERY scenario,
    alpha / beta to 1e-8 -- no near-tie exemption."""
    from oracle import cpu
    from sqlp_amd import smps, twosd
    inst = I.load("storm")
    ctx = twosd.SDContext(inst["sp2"], inst["sto"])
    x = I.x_ev("storm")
    ctx.compute_basis(x, smps.mean_values(inst["sto"]))
    src = twosd.sdEpigraph(ctx, 1.0, 0.0)
    twosd.add_scenarios(src, I.sample("storm", 16384, 41))
    _, st, _ = twosd.solve_push(src, x, 0, 16384)
    assert (st == 0).all()
    V = twosd.sdDualVertexSet(ctx)
    assert len(V) >= 256
    N = 4096
    vals = I.sample("storm", N, 43)
    epi = twosd.sdEpigraph(ctx, 1.0, 0.0)
    twosd.add_scenarios(epi, vals)
    sp = I.load("storm")["osp2"]
    Vm = V.matrix()
    scores = (Vm @ (sp.r - sp.T @ x))[None, :] + (vals - sp.r[ctx.rows]) @ Vm[:, ctx.rows].T
    part = np.partition(scores, -2, axis=1)[:, -2:]
    ties = int(((part.max(1) - part.min(1)) <= 1e-9 * (1 + np.abs(part.max(1)))).sum())
    assert ties > N // 4, ties                  # the case this test is about
    for tie_rel in (0.0, 1e-12):
        a, b, omv, oma = cpu.build_cut(sp.r, sp.T, x, Vm, ctx.rows, vals - sp.r[ctx.rows], np.ones(N), tie_rel=tie_rel,
                                       nthreads=8)
        got = {}
        # dominated twins left out of the argmax (default) and kept in it: the same picks, bit for bit
        for twins in ("1", "0"):
            with _env("TWOSD_CUT_TWINS", twins):
                cut, mv, ma = twosd._build_cut(epi, x, tie_rel, want_argmax=True)
                got[twins] = (cut, mv, ma, ctx.cut_stats())
            assert (ma == oma).all(), (tie_rel, twins, ties, int((ma != oma).sum()))
            np.testing.assert_allclose(mv, omv, rtol=1e-12, atol=1e-9)
            assert cut.alpha == pytest.approx(a, rel=1e-8, abs=1e-8)
            np.testing.assert_allclose(cut.beta, b, rtol=1e-8, atol=1e-8 * (1 + np.abs(b).max()))
        (c1, mv1, ma1, st1), (c0, mv0, ma0, st0) = got["1"], got["0"]
        # the same picks; the cut sums add the re-decided rows in other waves' partials (more rows
        # are re-decided with the twins kept), so alpha / beta agree to rounding, not bit for bit;
        # max_val is the MFMA score where a row was decided without the fixup, the restated score
        # where it was re-decided
        assert np.array_equal(ma1, ma0)
        assert c1.alpha == pytest.approx(c0.alpha, rel=1e-13)
        np.testing.assert_allclose(c1.beta, c0.beta, rtol=1e-13, atol=1e-13 * (1 + np.abs(c0.beta).max()))
        np.testing.assert_allclose(mv1, mv0, rtol=1e-12)
        assert st1[3] > 0 and st0[3] == 0, (st1, st0)      # storm's V has twins at x_EV
        assert st1[0] < st0[0], (st1, st0)                 # fewer scenarios re-decided without them


def test_cut_many_exact_ties_overflow_the_logs():
    """97 vertices with bit-identical scores at every scenario (a real dual plus copies that
    differ only in a row whose r - T x and deltas are exactly zero).  Left in the argmax, each
    lane group's candidate log overflows (~24 > 16 entries), so the fixup re-scans every vertex in the
    restatement's order; by default they are left out as dominated twins.  Either way the pick is
    the lowest index, as the strict '>' of subprob.jl:156 keeps the first maximum."""
    from oracle import cpu
    from sqlp_amd import twosd
    ctx, x, V0 = _setup("transship", 512)
    sp = I.load("transship")["osp2"]
    base = sp.r - sp.T @ x
    free = [i for i in range(len(sp.r)) if sp.r[i] == 0.0 and not sp.T[i].any() and i not in set(ctx.rows.tolist())]
    assert free, "no row with r - T x identically zero"
    i0 = free[0]
    assert base[i0] == 0.0
    Vm0 = V0.matrix()
    N = 3000
    vals = I.sample("transship", N, 47)
    # the vertex most scenarios pick, copied 96 times ahead of the rest
    _, _, _, oma0 = cpu.build_cut(sp.r, sp.T, x, Vm0, ctx.rows, vals - sp.r[ctx.rows], np.ones(N), tie_rel=0.0)
    top = int(np.bincount(oma0).argmax())
    copies = np.repeat(Vm0[top][None, :], 97, axis=0)
    copies[1:, i0] += np.arange(1, 97, dtype=np.float64)
    V = twosd.sdDualVertexSet(ctx)          # the context's one set (V0): rebuilt with the copies first
    V.clear()
    V.push_batch(np.vstack([copies, Vm0]))
    assert len(V) == 96 + len(Vm0)                      # copies[0] is Vm0[top] itself
    epi = twosd.sdEpigraph(ctx, 1.0, 0.0)
    twosd.add_scenarios(epi, vals)
    Vm = V.matrix()
    for tie_rel in (0.0, 1e-12):
        a, b, omv, oma = cpu.build_cut(sp.r, sp.T, x, Vm, ctx.rows, vals - sp.r[ctx.rows], np.ones(N), tie_rel=tie_rel)
        assert (oma == 0).sum() >= (oma0 == top).sum(), (np.bincount(oma)[:45].tolist(), int((oma0 == top).sum()),
                                                         bool(np.array_equal(Vm[0], Vm0[top])), float(np.abs(Vm[1:97, i0] - Vm0[top, i0]).max()))
        # the copies' PK rows are the original's, so by default they are dominated twins left out of
        # the argmax; with TWOSD_CUT_TWINS=0 they stay in and every log of a scenario the copied
        # vertex wins overflows: the fixup re-scans every vertex
        for twins in ("1", "0"):
            with _env("TWOSD_CUT_TWINS", twins):
                cut, mv, ma = twosd._build_cut(epi, x, tie_rel, want_argmax=True)
                st = ctx.cut_stats()
            assert (ma == oma).all(), (tie_rel, twins, int((ma != oma).sum()))
            assert cut.alpha == pytest.approx(a, rel=1e-8, abs=1e-8)
            np.testing.assert_allclose(cut.beta, b, rtol=1e-8, atol=1e-8 * (1 + np.abs(b).max()))
            if twins == "1":
                assert st[3] >= 96, st
            else:
                assert st[3] == 0 and st[2] > 0, st


def test_cut_after_truncate_and_different_pushes():
    """The cut keeps its per-vertex rows (PK, twin links) across cuts; truncating V and pushing
    other vectors must refresh exactly the rows past the truncation: the cut after
    truncate + push equals the C oracle on the new V (and a cut on a fresh context)."""
    from oracle import cpu
    from sqlp_amd import twosd
    ctx, x, V = _setup("ssn", nv_src=600, seed=3)
    sp = I.load("ssn")["osp2"]
    N = 2000
    vals = I.sample("ssn", N, seed=61)
    epi = twosd.sdEpigraph(ctx, 1.0, 0.0)
    twosd.add_scenarios(epi, vals)
    twosd._build_cut(epi, x, 0.0, want_argmax=True)          # rows of the first V built
    n0 = len(V)
    V.truncate(n0 // 2)
    _, _, pis, st = ctx.solve_values(x, I.sample("ssn", 400, seed=62), want_pi=True)
    V.push_batch(pis[st == 0])
    assert len(V) > n0 // 2
    Vm = V.matrix()
    for tie_rel in (0.0, 1e-12):
        cut, mv, ma = twosd._build_cut(epi, x, tie_rel, want_argmax=True)
        a, b, omv, oma = cpu.build_cut(sp.r, sp.T, x, Vm, ctx.rows, vals - sp.r[ctx.rows], np.ones(N), tie_rel=tie_rel)
        assert (ma == oma).all(), (tie_rel, int((ma != oma).sum()))
        assert cut.alpha == pytest.approx(a, rel=1e-8, abs=1e-8)
        np.testing.assert_allclose(cut.beta, b, rtol=1e-8, atol=1e-8 * (1 + np.abs(b).max()))


def test_cut_storm_twins_with_vertex_split_tail():
    """storm at x_EV with its twin-rich V (the duals of 16,384 scenarios solved there) over 100,000
    scenarios: 782 tiles on the persistent grid leave a vertex-split tail, so tail rows are merged
    across ranges and re-decided from the range logs, with the dominated twins left out of the MFMA
    pass.  max_arg equal to the C oracle for EVERY scenario, alpha / beta to 1e-8."""
    from oracle import cpu
    from sqlp_amd import smps, twosd
    inst = I.load("storm")
    ctx = twosd.SDContext(inst["sp2"], inst["sto"])
    x = I.x_ev("storm")
    ctx.compute_basis(x, smps.mean_values(inst["sto"]))
    src = twosd.sdEpigraph(ctx, 1.0, 0.0)
    twosd.add_scenarios(src, I.sample("storm", 16384, 41))
    _, st, _ = twosd.solve_push(src, x, 0, 16384)
    assert (st == 0).all()
    V = twosd.sdDualVertexSet(ctx)
    N = 100_000
    vals = I.sample("storm", N, 67)
    epi = twosd.sdEpigraph(ctx, 1.0, 0.0)
    twosd.add_scenarios(epi, vals)
    sp = inst["osp2"]
    Vm = V.matrix()
    cut, mv, ma = twosd._build_cut(epi, x, 0.0, want_argmax=True)
    assert ctx.cut_stats()[3] > 0                                  # twins left out
    a, b, omv, oma = cpu.build_cut(sp.r, sp.T, x, Vm, ctx.rows, vals - sp.r[ctx.rows], np.ones(N), tie_rel=0.0,
                                   nthreads=8)
    assert (ma == oma).all(), int((ma != oma).sum())
    np.testing.assert_allclose(mv, omv, rtol=1e-12, atol=1e-9)
    assert cut.alpha == pytest.approx(a, rel=1e-8, abs=1e-8)
    np.testing.assert_allclose(cut.beta, b, rtol=1e-8, atol=1e-8 * (1 + np.abs(b).max()))


def test_cut_log_offset_guard_and_empty_epigraph_stats():
    """The argmax's candidate-log offsets are 32-bit: a cut needing more log slots than that is
    refused with TWOSD_E_UNSUPPORTED instead of wrapping (limit lowered by the TWOSD_CUT_LOG_MAX
    test hook), and the same cut runs once the limit allows it.  A cut over an epigraph with no
    scenarios reports no fixup counters (not the previous cut's)."""
    from sqlp_amd import twosd
    from sqlp_amd._lib import TwoSDError
    ctx, x, V = _setup("ssn", 512)
    epi = twosd.sdEpigraph(ctx, 1.0, 0.0)
    twosd.add_scenarios(epi, I.sample("ssn", 5000, 71))
    with _env("TWOSD_CUT_LOG_MAX", "4096"):
        with pytest.raises(TwoSDError) as ei:
            twosd.build_sasa_cut(epi, x, V)
        assert ei.value.code == -5 and "32-bit" in str(ei.value)
    cut = twosd.build_sasa_cut(epi, x, V)
    assert np.isfinite(cut.alpha)
    empty = twosd.sdEpigraph(ctx, 1.0, 0.0)
    c0 = twosd.build_sasa_cut(empty, x, V)
    assert c0.alpha == 0.0 and not c0.beta.any()
    assert ctx.cut_stats()[:3] == (0, 0, 0)


@pytest.mark.parametrize("name,N", [("storm", 6000), ("ssn", 5000)])
def test_cut_fp32_pass_equals_fp64_pass(name, N):
    """The fp32 MFMA pass (default) and the fp64 one (TWOSD_CUT_F32=0) decide the same rows: both
    give the C oracle's pick for every scenario under both tie rules; alpha / beta to 1e-8 of the
    oracle.  storm at x_EV with V built there (twin-rich, many exact ties)."""
    from oracle import cpu
    from sqlp_amd import smps, twosd
    inst = I.load(name)
    ctx = twosd.SDContext(inst["sp2"], inst["sto"])
    x = I.x_ev(name)
    ctx.compute_basis(x, smps.mean_values(inst["sto"]))
    src = twosd.sdEpigraph(ctx, 1.0, 0.0)
    twosd.add_scenarios(src, I.sample(name, 8192, 41))
    _, st, _ = twosd.solve_push(src, x, 0, 8192)
    assert (st == 0).all()
    V = twosd.sdDualVertexSet(ctx)
    vals = I.sample(name, N, 43)
    w = np.random.default_rng(9).uniform(0.5, 1.5, size=N)
    epi = twosd.sdEpigraph(ctx, 1.0, 0.0)
    twosd.add_scenarios(epi, vals, w)
    sp = inst["osp2"]
    Vm = V.matrix()
    for tie_rel in (0.0, 1e-12):
        a, b, omv, oma = cpu.build_cut(sp.r, sp.T, x, Vm, ctx.rows, vals - sp.r[ctx.rows], w, tie_rel=tie_rel, nthreads=8)
        got = {}
        for f32 in ("1", "0"):
            with _env("TWOSD_CUT_F32", f32):
                cut, mv, ma = twosd._build_cut(epi, x, tie_rel, want_argmax=True)
                got[f32] = (cut, ctx.cut_pass())
            assert got[f32][1][0] == int(f32)
            assert (ma == oma).all(), (f32, tie_rel, int((ma != oma).sum()))
            np.testing.assert_allclose(mv, omv, rtol=1e-12, atol=1e-9)
            assert cut.alpha == pytest.approx(a, rel=1e-8, abs=1e-8)
            np.testing.assert_allclose(cut.beta, b, rtol=1e-8, atol=1e-8 * (1 + np.abs(b).max()))
        assert got["1"][1][1] > got["0"][1][1] > 0.0          # the fp32 band is the wider one


def test_cut_operands_past_fp32_envelope_run_the_fp64_pass():
    """A vertex whose entries on the random rows are ~1e32 puts the fp32 operands' products past
    the pass's envelope: the cut runs the fp64 pass (decided on the device) and still gives the
    oracle's picks."""
    from oracle import cpu
    from sqlp_amd import twosd
    ctx, x, V0 = _setup("ssn", 300)
    Vm0 = V0.matrix()
    big = Vm0[1].copy()
    big[ctx.rows] *= 1e32
    V0.push_batch(big[None, :])
    Vm = V0.matrix()
    N = 2000
    vals = I.sample("ssn", N, 73)
    epi = twosd.sdEpigraph(ctx, 1.0, 0.0)
    twosd.add_scenarios(epi, vals)
    sp = I.load("ssn")["osp2"]
    cut, mv, ma = twosd._build_cut(epi, x, 0.0, want_argmax=True)
    assert ctx.cut_pass()[0] == 0
    a, b, omv, oma = cpu.build_cut(sp.r, sp.T, x, Vm, ctx.rows, vals - sp.r[ctx.rows], np.ones(N), tie_rel=0.0, nthreads=8)
    assert (ma == oma).all(), int((ma != oma).sum())
    assert cut.alpha == pytest.approx(a, rel=1e-8, abs=1e-8)

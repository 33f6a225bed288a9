"""Multi-rank path on CPU (world_size 2, gloo): scenario sharding, the cut-partial
all-reduce (exact uint64 fixed-point vertex histogram + fp64 sums) and the ordered
vertex all-gather of sqlp_amd.dist, checked against single-rank results.  Per-rank
compute is emulated with the oracle (no GPU needed); the collectives are the product's."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import twosd_ref
from sqlp_amd import dist as sdist


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _problem():
    rng = np.random.default_rng(3)
    m, n1, k, nv, N = 12, 4, 5, 9, 37
    rows = np.array([0, 3, 5, 7, 11])
    cols = np.array([-1, -1, 2, -1, 0])          # two T-matrix elements, three RHS elements
    r = rng.normal(size=m)
    T = rng.normal(size=(m, n1))
    V = np.round(rng.normal(size=(nv, m)), 3)
    dv = rng.normal(size=(N, k))
    w = rng.uniform(0.5, 2.0, size=N)
    x = rng.normal(size=n1)
    return m, n1, k, rows, cols, r, T, V, dv, w, x


def _partial(lo, hi, total_w):
    """Restatement of twosd_cut_partial's semantics for scenarios [lo, hi)."""
    m, n1, k, rows, cols, r, T, V, dv, w, x = _problem()
    coef = np.where(cols < 0, 1.0, -x[np.maximum(cols, 0)])
    base = V @ (r - T @ x)
    hist = np.zeros(V.shape[0], dtype=np.int64)
    sums = np.zeros(k + 1)
    for s in range(lo, hi):
        sc = base + V[:, rows] @ (coef * dv[s])
        a = int(np.argmax(sc))
        p = w[s] / total_w
        hist[a] += int(np.rint(p * 2.0 ** 62))
        sums[0] += p * sc[a]
        sums[1:] += p * V[a, rows] * dv[s]
    return hist, sums


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    m, n1, k, rows, cols, r, T, V, dv, w, x = _problem()
    N = dv.shape[0]
    lo, hi = sdist.shard_range(N, rank, world)
    h, s = _partial(lo, hi, w.sum())
    ht, st = torch.from_numpy(h.copy()), torch.from_numpy(s.copy())
    sdist.allreduce_cut_partials(ht, st)
    alpha, beta = sdist.finalize_from_partials(ht.numpy(), st.numpy(), V, r, T, cols)
    # ordered all-gather of per-rank new vertices (variable counts)
    mine = torch.arange(3 * (rank + 1) * m, dtype=torch.float64).reshape(-1, m) + 1000 * rank
    allrows = sdist.allgather_rows_ordered(mine)
    ev = sdist.sum_in_rank_order(0.1 * (rank + 1))   # evaluate(): shards' partials in rank order
    out[rank] = (ht.numpy(), st.numpy(), alpha, beta, allrows.numpy(), ev)
    dist.destroy_process_group()


def test_shard_ranges_cover():
    for N in (0, 1, 7, 1000, 1_000_000):
        for G in (1, 2, 3, 8):
            rs = [sdist.shard_range(N, g, G) for g in range(G)]
            assert rs[0][0] == 0 and rs[-1][1] == N
            assert all(rs[i][1] == rs[i + 1][0] for i in range(G - 1))
            assert max(b - a for a, b in rs) - min(b - a for a, b in rs) <= 1


def test_two_rank_cut_and_gather():
    port = _free_port()
    with mp.Manager() as mgr:
        out = mgr.dict()
        mp.spawn(_worker, args=(2, port, out), nprocs=2, join=True)
        res = dict(out)
    m, n1, k, rows, cols, r, T, V, dv, w, x = _problem()
    h1, s1 = _partial(0, dv.shape[0], w.sum())
    for rank in (0, 1):
        h, s, alpha, beta, allrows, ev = res[rank]
        assert ev == 0.0 + 0.1 + 0.2
        assert (h == h1).all()                         # exact: fixed point, order independent
        np.testing.assert_allclose(s, s1, rtol=1e-13, atol=1e-14)
        a1, b1 = sdist.finalize_from_partials(h1, s1, V, r, T, cols)
        assert alpha == pytest.approx(a1, rel=1e-12) and np.allclose(beta, b1, rtol=1e-12)
        assert allrows.shape[0] == 3 * 1 + 3 * 2
        assert allrows[0, 0] == 0 and allrows[3, 0] == 1000
    assert np.array_equal(res[0][4], res[1][4])
    # the sharded cut equals the reference-order build_sasa_cut on the whole batch
    coef_ref = twosd_ref.Coefficients(type("SP", (), dict(
        r=r, T=T, W=np.zeros((len(r), 1)), last_names=[f"x{j}" for j in range(n1)],
        row_names=[f"r{i}" for i in range(len(r))]))())
    pos = [("RHS" if c < 0 else f"x{c}", f"r{i}") for i, c in zip(rows, cols)]
    deltas = []
    for s in range(dv.shape[0]):
        sc = [(p, (r[i] if c < 0 else T[i, c]) + dv[s, e]) for e, (p, i, c) in enumerate(zip(pos, rows, cols))]
        deltas.append(twosd_ref.delta_coefficients(coef_ref, sc))
    a_ref, b_ref, wm, _, _ = twosd_ref.build_sasa_cut(coef_ref, deltas, w, x, twosd_ref.DualVertexSet(list(V)))
    assert res[0][2] == pytest.approx(a_ref, rel=1e-10)
    np.testing.assert_allclose(res[0][3], b_ref, rtol=1e-10, atol=1e-12)


def test_ordered_vertex_merge_equals_sequential_push():
    """Each rank dedups locally, the locally-new rows are gathered in rank order and pushed:
    the final set equals a sequential push! of all duals in (rank, index) order."""
    rng = np.random.default_rng(9)
    base = np.round(rng.normal(size=(6, 5)), 2)
    per_rank = [base[rng.integers(0, 6, size=8)] for _ in range(2)]
    V0 = twosd_ref.DualVertexSet(list(base[:2]))
    seq = twosd_ref.DualVertexSet(list(base[:2]))
    for blk in per_rank:
        for v in blk:
            seq.push(v)
    merged = twosd_ref.DualVertexSet(list(base[:2]))
    for blk in per_rank:                      # allgather order = rank order
        local = twosd_ref.DualVertexSet(list(base[:2]))
        new_rows = []
        for v in blk:
            before = len(local)
            local.push(v)
            if len(local) > before:
                new_rows.append(v)
        for v in new_rows:
            merged.push(v)
    assert len(merged) == len(seq)
    assert all(np.array_equal(a, b) for a, b in zip(merged.data, seq.data))


class _FakeCutCtx:
    """Stand-in for SDContext's cut partial / finalize (the oracle's semantics, no GPU): writes
    this rank's partials into the exchange's buffers through their data pointers, as the
    library does, and finalizes from them."""

    def __init__(self, lo, hi):
        self.lo, self.hi = lo, hi
        self.prob = _problem()

    def cut_partial_len(self):
        m, n1, k, rows, cols, r, T, V, dv, w, x = self.prob
        return V.shape[0], k + 1

    def cut_partial(self, epi, x, tie_rel, total_weight, hist_ptr, sums_ptr):
        import ctypes as C
        h, s = _partial(self.lo, self.hi, total_weight)
        np.ctypeslib.as_array((C.c_int64 * h.size).from_address(hist_ptr))[:] = h
        np.ctypeslib.as_array((C.c_double * s.size).from_address(sums_ptr))[:] = s

    def cut_finalize(self, x, hist_ptr, sums_ptr):
        import ctypes as C
        m, n1, k, rows, cols, r, T, V, dv, w, xx = self.prob
        h = np.ctypeslib.as_array((C.c_int64 * V.shape[0]).from_address(hist_ptr)).copy()
        s = np.ctypeslib.as_array((C.c_double * (k + 1)).from_address(sums_ptr)).copy()
        return sdist.finalize_from_partials(h, s, V, r, T, cols)


def _extra_worker(rank, world, port, mismatch, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        m, n1, k, rows, cols, r, T, V, dv, w, x = _problem()
        lo, hi = sdist.shard_range(dv.shape[0], rank, world)
        ex = sdist.CutExchange(_FakeCutCtx(lo, hi), torch.device("cpu"))
        a1, b1 = ex.build_cut(0, x, w.sum(), 0.0, verify=False)
        extra = [1.5 * (rank + 1), 0.25 * rank]
        a2, b2, es = ex.build_cut(0, x, w.sum(), 0.0, verify=False, extra=extra)
        # the vertex-set check riding in the fp64 all-reduce (size + fingerprint pieces)
        row = np.array([9.0, 11.0, 2.0, 65535.0, 7.0])
        if mismatch and rank == 1:
            row[3] -= 1.0
        sdist._vertex_check_row = lambda ctx: row.copy()
        try:
            a3, b3, es3 = ex.build_cut(0, x, w.sum(), 0.0, verify=True, extra=extra)
            chk = "passed"
        except RuntimeError:
            a3, b3, es3, chk = None, None, None, "raised"
        out[rank] = (a1, b1, a2, b2, es, a3, b3, es3, chk)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("mismatch", [False, True])
def test_cut_exchange_extra_and_vertex_check(mismatch):
    """CutExchange.build_cut with extra fp64 values (bench: the incumbent objective's sum w obj and
    sum w) in the cut's all-reduce: alpha / beta bit-identical to the call without extra, the
    extra slots the ranks' totals; the vertex-set check in the same all-reduce passes when the
    sets agree and raises on every rank when they do not."""
    port = _free_port()
    with mp.get_context("spawn").Manager() as mgr:
        out = mgr.dict()
        mp.start_processes(_extra_worker, args=(2, port, mismatch, out), nprocs=2, join=True, start_method="spawn")
        res = dict(out)
    m, n1, k, rows, cols, r, T, V, dv, w, x = _problem()
    want_extra = np.array([1.5 + 3.0, 0.25])
    for rnk in (0, 1):
        a1, b1, a2, b2, es, a3, b3, es3, chk = res[rnk]
        assert a1 == a2 and np.array_equal(b1, b2)
        np.testing.assert_array_equal(es, want_extra)
        if mismatch:
            assert chk == "raised"
        else:
            assert chk == "passed" and a3 == a1 and np.array_equal(b3, b1)
            np.testing.assert_array_equal(es3, want_extra)
    assert res[0][0] == res[1][0]

"""Scenario data-parallelism across GPUs (one process per GPU, torch.distributed).

The reference is single-process (no MPI/NCCL; the comments at
algorithm.jl:7,10-11 and cell.jl:25 only anticipate per-epigraph parallelism).  Here the
hot path shards naturally by scenario:
  * LP solves and argmax are per scenario against a replicated template / vertex set;
    rank g owns the contiguous range shard_range(N, g, G).
  * build_sasa_cut needs ONE exchange: the vertex-weight histogram (uint64 fixed point,
    summed exactly, so every rank count gives bit-identical h) and k+1 fp64 sums,
    all-reduced over RCCL (backend "nccl") -- a few KB per cut.
  * vertex-set growth (push_sharded): every rank dedups its new duals locally, then the
    locally-new rows are all-gathered and pushed in (rank, local index) order, so every rank
    holds the same ordered set (the order decides argmax ties); every cut all-reduce checks
    size + fingerprint across ranks inside its own fp64 sums (CutExchange.build_cut: no extra
    collective, all ranks raise alike before the histogram all-reduce).
The collectives are plain torch.distributed calls on tensors, so the same code runs on
CPU tensors with gloo (tests) and on HIP tensors with RCCL (bench).
"""
from __future__ import annotations

import numpy as np
import torch
import torch.distributed as dist


def world():
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def shard_range(N: int, rank: int, world_size: int):
    """Contiguous scenario range [lo, hi) of `rank`."""
    return (N * rank) // world_size, (N * (rank + 1)) // world_size


def allreduce_cut_partials(hist: torch.Tensor, sums: torch.Tensor):
    """Sum the per-rank cut partials in place: hist (int64 fixed point, exact) and sums
    (fp64).  No-op on a single rank."""
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(hist, op=dist.ReduceOp.SUM)
        dist.all_reduce(sums, op=dist.ReduceOp.SUM)
    return hist, sums


def allgather_rows_ordered(rows: torch.Tensor) -> torch.Tensor:
    """Concatenate every rank's (n_r x m) rows in rank order (variable n_r): one fixed all-gather
    of the counts (one host synchronisation), then the rows padded to the longest."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return rows
    G = dist.get_world_size()
    counts = [int(c) for c in _gather_fixed(np.array([rows.shape[0]], dtype=np.int64), rows.device)[:, 0]]
    mx = max(counts)
    if mx == 0:
        return rows[:0]
    pad = torch.zeros((mx, rows.shape[1]), dtype=rows.dtype, device=rows.device)
    pad[: rows.shape[0]] = rows
    bufs = [torch.zeros_like(pad) for _ in range(G)]
    dist.all_gather(bufs, pad)
    return torch.cat([b[:c] for b, c in zip(bufs, counts)], dim=0)


def sum_in_rank_order(value: float) -> float:
    """All-gather one fp64 per rank and sum in rank order (identical on every rank,
    independent of the reduction tree).  Single rank: the value itself."""
    if not (dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1):
        return float(value)
    t = torch.tensor([float(value)], dtype=torch.float64)
    if dist.get_backend() == "nccl":
        t = t.cuda()
    parts = [torch.zeros_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(parts, t)
    acc = 0.0
    for p in parts:
        acc += float(p.item())
    return acc


def evaluate_sharded(ctx, first_stage_cost, x, N, seed):
    """evaluate(sp1, sp2, sto, x; N) (smps_routines.jl:67-82) with the N device-drawn
    scenarios of stream `seed` split over the ranks: c'x + sum of the shards' in-order
    partial sums, combined in rank order."""
    from . import twosd
    rank, G = world()
    lo, hi = shard_range(N, rank, G)
    s2 = twosd.evaluate_sampled(ctx, np.zeros(len(x)), x, N, seed, lo, hi - lo)
    return float(np.dot(first_stage_cost, x)) + sum_in_rank_order(s2)


class CutExchange:
    """Device buffers of the per-cut exchange of one context, allocated once and regrown only
    when the vertex set grows (no per-cut allocation)."""

    def __init__(self, ctx, device):
        self.ctx = ctx
        self.device = device
        self.hist = None
        self.sums = None

    def _buffers(self, n_extra=0):
        n_u64, n_f64 = self.ctx.cut_partial_len()
        if self.hist is None or self.hist.numel() < n_u64:
            self.hist = torch.zeros(max(n_u64, 1024), dtype=torch.int64, device=self.device)
            self._sync()
        if self.sums is None or self.sums.numel() < n_f64 + n_extra:
            self.sums = torch.zeros(max(n_f64 + n_extra, 256), dtype=torch.float64, device=self.device)
            self._sync()     # torch's fill must land before the library's stream touches the buffer
        return self.hist[:n_u64], self.sums[:n_f64 + n_extra], n_f64

    def _sync(self):
        if self.hist is not None and self.hist.is_cuda:
            torch.cuda.synchronize(self.device)

    def build_cut(self, epi, x, total_weight, tie_rel, verify=True, extra=None):
        """build_sasa_cut over the scenarios of every rank: local partial on this GPU (the
        library zero-fills and writes the buffers on its stream, synchronously), all-reduce,
        identical finalize on every rank.  Returns (alpha, beta), or (alpha, beta, sums of
        `extra`) when extra (a few fp64 per rank, e.g. the incumbent objective's sum_s w_s obj_s
        and sum_s w_s) is given: those travel in the same all-reduce as the cut's fp64 sums.
        verify: the vertex sets must agree (the histogram adds by vertex index).  The check rides
        in the fp64 all-reduce, which runs before the histogram's: each rank adds v and v^2 for
        v = |V| and the four 16-bit pieces of its set fingerprint; the sets agree iff every sum
        equals G v and G v^2 (equality in Cauchy-Schwarz), which every rank then sees alike --
        all raise, or none, and no collective of a different length is entered."""
        G = world()[1]
        n_extra = 0 if extra is None else len(extra)
        chk = _vertex_check_row(self.ctx) if (verify and G > 1) else None
        n_chk = 0 if chk is None else 2 * len(chk)
        hist, sums, n_f64 = self._buffers(n_extra + n_chk)
        self.ctx.cut_partial(epi, x, tie_rel, total_weight, hist.data_ptr(), sums.data_ptr())
        tail = []
        if n_extra:
            tail.append(np.asarray(extra, dtype=np.float64))
        if n_chk:
            tail.append(np.concatenate([chk, chk * chk]))
        if tail:
            sums[n_f64:] = torch.tensor(np.concatenate(tail), device=sums.device)
        if G > 1:
            dist.all_reduce(sums, op=dist.ReduceOp.SUM)
            if n_chk:
                got = sums[n_f64 + n_extra:].cpu().numpy()
                want = G * np.concatenate([chk, chk * chk])
                if not np.array_equal(got, want):
                    raise RuntimeError(f"vertex sets differ across ranks: this rank (size, fingerprint pieces) = "
                                       f"{chk.astype(np.int64).tolist()}, sums over {G} ranks = {got[:len(chk)].tolist()}")
            dist.all_reduce(hist, op=dist.ReduceOp.SUM)
        self._sync()         # the collective runs on torch / RCCL streams, finalize on the library's
        cut = self.ctx.cut_finalize(x, hist.data_ptr(), sums.data_ptr())
        if extra is None:
            return cut
        return cut[0], cut[1], sums[n_f64:n_f64 + n_extra].cpu().numpy()


def build_cut_sharded(ctx, epi, x, total_weight, tie_rel, device, verify=True, extra=None):
    """build_sasa_cut over the scenarios of every rank (one CutExchange per context); `extra`:
    see CutExchange.build_cut."""
    ex = getattr(ctx, "_cut_exchange", None)
    if ex is None:
        ex = ctx._cut_exchange = CutExchange(ctx, device)
    return ex.build_cut(epi, x, total_weight, tie_rel, verify=verify, extra=extra)


def _vertex_check_row(ctx) -> np.ndarray:
    """(|V|, the fingerprint's four 16-bit pieces) as fp64: integers whose squares and sums over
    any rank count stay exact."""
    from .twosd import sdDualVertexSet
    V = sdDualVertexSet(ctx)
    fp = int(V.fingerprint()) & ((1 << 64) - 1)
    return np.array([len(V)] + [(fp >> (16 * i)) & 0xFFFF for i in range(4)], dtype=np.float64)


def check_vertex_sets_agree(ctx):
    """Raise unless every rank holds the same ordered vertex set (size + order-dependent
    fingerprint, twosd_dvs_fingerprint): the histogram all-reduce sums by vertex index, so
    ranks with different sets would hang (different lengths) or add unrelated vertices."""
    rank, G = world()
    if G == 1:
        return
    from .twosd import sdDualVertexSet
    V = sdDualVertexSet(ctx)
    fp = V.fingerprint()
    mine = torch.tensor([len(V), fp - (1 << 64) if fp >= (1 << 63) else fp], dtype=torch.int64)
    if dist.get_backend() == "nccl":
        mine = mine.cuda()
    parts = [torch.zeros_like(mine) for _ in range(G)]
    dist.all_gather(parts, mine)
    rows = [tuple(int(v) for v in p.cpu().tolist()) for p in parts]
    if any(r != rows[0] for r in rows):
        raise RuntimeError(f"vertex sets differ across ranks (size, fingerprint) = {rows}")


def push_sharded(V, pis_local: np.ndarray) -> int:
    """Vertex-set growth across ranks (exchange 2): each rank dedups its own duals against
    the common set, rolls its set back, and every rank pushes the all-gathered locally-new
    rows in (rank, index) order -- the set equals a sequential push! of all ranks' duals in
    rank order on every rank.  Returns the new size."""
    n0 = len(V)
    pis_local = np.ascontiguousarray(np.atleast_2d(pis_local), dtype=np.float64)
    if pis_local.shape[0]:
        V.push_batch(pis_local)
    new_rows = V.matrix(n0) if len(V) > n0 else np.zeros((0, V.ctx.m))
    rank, G = world()
    if G == 1:
        return len(V)
    V.truncate(n0)
    t = torch.from_numpy(new_rows)
    if dist.get_backend() == "nccl":
        t = t.cuda()
    allrows = allgather_rows_ordered(t).cpu().numpy()
    if allrows.shape[0]:
        V.push_batch(allrows)
    return len(V)


def select_refresh_bases(keys, counts, reps, rank_of, max_pool):
    """Global selection of a distributed pool refresh, identical on every rank.  keys / counts /
    reps / rank_of: the distinct optimal bases of every rank's training slice, concatenated in
    rank order (within a rank ascending by first scenario, as twosd_refresh_train lists them).
    A basis seen by several ranks counts the sum of their counts and belongs to the rank of its
    first occurrence.  The max_pool - 1 most frequent, ties by first occurrence in (rank,
    scenario) order -- the single-rank refresh's stable sort over all training scenarios.
    Returns (owner rank, owner's first scenario) of the picks, in pool order."""
    import ctypes
    from ._lib import check, load
    keys = np.ascontiguousarray(keys, dtype=np.uint64)
    n = int(keys.size)
    if n == 0 or max_pool <= 1:
        return np.zeros(0, dtype=np.int64), np.zeros(0, dtype=np.int64)
    cnt = np.ascontiguousarray(counts, dtype=np.int64)
    rp = np.ascontiguousarray(reps, dtype=np.int64)
    rk = np.ascontiguousarray(rank_of, dtype=np.int32)
    k = min(n, max_pool - 1)
    owner = np.zeros(k, dtype=np.int64)
    rep = np.zeros(k, dtype=np.int64)
    npick = ctypes.c_int(0)
    ptr = lambda a: a.ctypes.data_as(ctypes.c_void_p)
    check(load().twosd_select_refresh_bases(ptr(keys), ptr(cnt), ptr(rp), ptr(rk), n, int(max_pool), ptr(owner), ptr(rep),
                                            ctypes.byref(npick)))
    return owner[:npick.value], rep[:npick.value]


def _select_refresh_bases_np(keys, counts, reps, rank_of, max_pool):
    """numpy statement of select_refresh_bases (the tests check the native one against it)."""
    keys = np.asarray(keys, dtype=np.uint64)
    if keys.size == 0 or max_pool <= 1:
        return np.zeros(0, dtype=np.int64), np.zeros(0, dtype=np.int64)
    _, first, inv = np.unique(keys, return_index=True, return_inverse=True)
    tot = np.bincount(inv.reshape(-1), weights=np.asarray(counts, dtype=np.float64)).astype(np.int64)
    order = np.lexsort((first, -tot))[: max_pool - 1]          # by -count, then first occurrence
    pick = first[order]
    return np.asarray(rank_of)[pick].astype(np.int64), np.asarray(reps)[pick].astype(np.int64)


def pack_positions(owner, G):
    """Source id of every pick in the gathered table: 1 + its position among all packs, packs
    in rank order, each pack in selection order (the primary is source 0)."""
    owner = np.asarray(owner, dtype=np.int64)
    if owner.size == 0:
        return np.zeros(0, dtype=np.int64)
    n_own = np.bincount(owner, minlength=G)
    base = 1 + np.concatenate([[0], np.cumsum(n_own)[:-1]])
    order = np.argsort(owner, kind="stable")
    rank_in = np.empty(owner.size, dtype=np.int64)
    rank_in[order] = np.arange(owner.size) - np.repeat(np.cumsum(n_own) - n_own, n_own)
    return base[owner] + rank_in


def _allgather_1d(arr: np.ndarray, device=None):
    """Rank-order concatenation of every rank's 1-D array (variable lengths) and the length of
    each part.  Host arrays; over RCCL they travel as device tensors."""
    G = dist.get_world_size()
    t = torch.from_numpy(np.ascontiguousarray(arr))
    nccl = dist.get_backend() == "nccl"
    if nccl:
        t = t.to(device)
    n = torch.tensor([t.numel()], dtype=torch.int64, device=t.device)
    ns = [torch.zeros_like(n) for _ in range(G)]
    dist.all_gather(ns, n)
    ns = [int(v.item()) for v in ns]
    pad = torch.zeros(max(max(ns), 1), dtype=t.dtype, device=t.device)
    pad[: t.numel()] = t
    bufs = [torch.zeros_like(pad) for _ in range(G)]
    dist.all_gather(bufs, pad)
    return np.concatenate([b[:k].cpu().numpy() for b, k in zip(bufs, ns)]), ns


def _gather_fixed(arr: np.ndarray, device=None) -> np.ndarray:
    """One all-gather of an equal-length int64 row per rank -> (G, len) host array.  Over RCCL a
    single all_gather_into_tensor of a device buffer, one host synchronisation."""
    G = dist.get_world_size()
    t = torch.from_numpy(np.ascontiguousarray(arr, dtype=np.int64))
    if dist.get_backend() == "nccl":
        t = t.to(device)
        out = torch.empty(G * t.numel(), dtype=torch.int64, device=device)
        dist.all_gather_into_tensor(out, t)
        return out.cpu().numpy().reshape(G, -1)
    parts = [torch.empty_like(t) for _ in range(G)]
    dist.all_gather(parts, t)
    return torch.stack(parts).numpy()


def _allreduce_i64(arr, device=None, op=None) -> np.ndarray:
    t = torch.tensor(np.asarray(arr, dtype=np.int64))
    if dist.get_backend() == "nccl":
        t = t.to(device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM if op is None else op)
    return t.cpu().numpy()


def exchange_training_bases(keys, counts, reps, lo, hi, ns, device=None):
    """Exchange 2 of refresh_sharded: every rank's distinct training bases (u64 keys, counts,
    first scenarios; ns[r] of them on rank r, known from the header exchange) and delta box in
    ONE all-gather of an int64 row padded to the longest rank.  Returns the rank-order
    concatenations and the union box."""
    G = dist.get_world_size()
    k = np.asarray(lo).size
    U = max(max(ns), 1)
    n = len(keys)
    row = np.zeros(3 * U + 2 * k, dtype=np.int64)
    row[:n] = np.asarray(keys, dtype=np.uint64).view(np.int64)
    row[U:U + n] = counts
    row[2 * U:2 * U + n] = reps
    row[3 * U:3 * U + k] = np.ascontiguousarray(lo, dtype=np.float64).view(np.int64)
    row[3 * U + k:] = np.ascontiguousarray(hi, dtype=np.float64).view(np.int64)
    g = _gather_fixed(row, device)
    all_keys = np.concatenate([g[r, :ns[r]] for r in range(G)]).view(np.uint64)
    all_counts = np.concatenate([g[r, U:U + ns[r]] for r in range(G)])
    all_reps = np.concatenate([g[r, 2 * U:2 * U + ns[r]] for r in range(G)])
    boxes = np.ascontiguousarray(g[:, 3 * U:]).view(np.float64).reshape(G, 2, k)
    return all_keys, all_counts, all_reps, boxes[:, 0].min(axis=0), boxes[:, 1].max(axis=0)


def refresh_training_cap(ctx, device=None) -> int:
    """The training pivot cap every rank uses (twosd_refresh_train_ex): the context's explicit
    setting, else twosd_pool_refresh's auto rule -- 3 x the mean pivots of the last batch of
    >= 4096 scenarios, at least 32 -- over every rank's last batch (one all-reduce of two int64),
    so all ranks train under the same cap whatever their own batches were.  0: none."""
    ps, pn = ctx.refresh_cap_stats()
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        ps, pn = (int(v) for v in _allreduce_i64([ps, pn], device))
    return ctx.training_cap(ps, pn)        # the native rule (setting, env, auto) on the global sums


def refresh_sharded(ctx, train_epi, x, first, count, max_pool, level1=0, ncand=0, device=None):
    """twosd_pool_refresh of the training scenarios of every rank (this rank: [first,
    first + count) of train_epi, the ranks' slices contiguous in rank order) -- the same pool on
    every rank, equal to one rank refreshing from all of them:
      0. one training pivot cap for all ranks (refresh_training_cap);
      1. each rank solves its slice under it (twosd_refresh_train_ex); exchange 1: a fixed header
         per rank (distinct bases, optimal training scenarios, slice size).  When fewer than half
         of ALL training scenarios ended optimal, every rank solves again uncapped (the
         single-rank rule, decided once from the global count);
      2. exchange 2: one all-gather of (keys, counts, first scenarios, delta box) padded to the
         longest rank; select_refresh_bases on every rank;
      3. each rank composes the picks it owns (twosd_refresh_build_local);
      4. exchange 3: the pack size (max) and the packs (one all_gather_into_tensor of device
         buffers); every rank assembles the pool (twosd_refresh_assemble; no pick on any rank:
         the current pool stays);
      5. the two-level candidate lists from every rank's picks (exchange 4: one fixed all-gather).
    Exchanges 1-4 are 5-6 collectives in all, each followed by one host synchronisation.
    A template the device build does not fit (TWOSD_E_UNSUPPORTED) or a primary basis failing
    the device checks (TWOSD_E_STATE) -- both the same on every rank -- falls back to a per-rank
    twosd_pool_refresh of the rank's own slice (pools then differ between ranks; only pivots
    depend on the pool).
    Returns (pool size, phase milliseconds)."""
    import time
    from ._lib import TwoSDError
    rank, G = world()
    t = [time.perf_counter()]
    cap = refresh_training_cap(ctx, device)
    keys, counts, reps, lo, hi, nopt = ctx.refresh_train_ex(train_epi, x, first, count, cap)
    t.append(time.perf_counter())
    k = lo.size
    if G == 1:
        if cap > 0 and 2 * nopt < count:
            keys, counts, reps, lo, hi, nopt = ctx.refresh_train_ex(train_epi, x, first, count, 0)
        all_keys, all_counts, all_reps, ns = keys, counts, reps, [len(keys)]
        box_lo, box_hi = lo, hi
        counts_r = [count]
    else:
        hdr = _gather_fixed([len(keys), nopt, count], device)
        if cap > 0 and 2 * int(hdr[:, 1].sum()) < int(hdr[:, 2].sum()):
            keys, counts, reps, lo, hi, nopt = ctx.refresh_train_ex(train_epi, x, first, count, 0)
            hdr = _gather_fixed([len(keys), nopt, count], device)
        ns = [int(v) for v in hdr[:, 0]]
        counts_r = [int(v) for v in hdr[:, 2]]
        all_keys, all_counts, all_reps, box_lo, box_hi = exchange_training_bases(keys, counts, reps, lo, hi, ns, device)
    rank_of = np.repeat(np.arange(G), ns)
    owner, orep = select_refresh_bases(all_keys, all_counts, all_reps, rank_of, max_pool)
    mine = orep[owner == rank]
    pos = pack_positions(owner, G)
    t.append(time.perf_counter())
    try:
        nbytes = ctx.refresh_build_local(mine)
    except TwoSDError as e:
        if e.code != -5:
            raise
        return _refresh_local_fallback(ctx, train_epi, x, first, count, max_pool, level1, ncand, t)
    t.append(time.perf_counter())
    try:
        if G == 1:
            buf = torch.empty(nbytes, dtype=torch.uint8, device=device)
            torch.cuda.synchronize(device)
            ctx.refresh_pack(buf.data_ptr())
            size = ctx.refresh_assemble(1, buf.data_ptr(), nbytes, pos, box_lo, box_hi)
        else:
            mx = int(_allreduce_i64([nbytes], device, dist.ReduceOp.MAX)[0])
            stride = (mx + 255) // 256 * 256
            buf = torch.empty(stride, dtype=torch.uint8, device=device)
            torch.cuda.synchronize(device)
            ctx.refresh_pack(buf.data_ptr())
            if dist.get_backend() == "nccl":
                out = torch.empty(G * stride, dtype=torch.uint8, device=device)
                dist.all_gather_into_tensor(out, buf)
                torch.cuda.synchronize(device)
            else:   # gloo (tests, rehearsal): through host memory
                parts = [torch.empty(stride, dtype=torch.uint8) for _ in range(G)]
                dist.all_gather(parts, buf.cpu())
                out = torch.cat(parts).to(device)
                torch.cuda.synchronize(device)
            size = ctx.refresh_assemble(G, out.data_ptr(), stride, pos, box_lo, box_hi)
    except TwoSDError as e:
        if e.code != -3 or "primary basis failed" not in str(e):
            raise
        return _refresh_local_fallback(ctx, train_epi, x, first, count, max_pool, level1, ncand, t)
    t.append(time.perf_counter())
    if level1 > 0 and ncand > 0 and size > level1:
        p1, pf = ctx.pool_candidate_picks(train_epi, x, first, count, level1)
        if G > 1:
            M = max(counts_r)
            row = np.zeros(2 * M, dtype=np.int64)
            row[:count] = p1
            row[M:M + count] = pf
            g = _gather_fixed(row, device)
            p1 = np.concatenate([g[r, :counts_r[r]] for r in range(G)])
            pf = np.concatenate([g[r, M:M + counts_r[r]] for r in range(G)])
        ctx.pool_set_candidates(level1, ncand, p1, pf)
    t.append(time.perf_counter())
    ms = dict(zip(("train", "select", "build", "exchange_assemble", "candidates"),
                  (1e3 * (b - a) for a, b in zip(t[:-1], t[1:]))))
    ms["kcap"] = cap
    return size, ms


def _refresh_local_fallback(ctx, train_epi, x, first, count, max_pool, level1, ncand, t):
    """The device pool build does not fit (the same on every rank): each rank refreshes alone
    from its own slice (twosd_pool_refresh composes on the host then)."""
    import time
    size = ctx.pool_refresh(train_epi, x, first, count, max_pool)
    if level1 > 0 and ncand > 0 and size > level1:
        ctx.pool_build_candidates(train_epi, x, first, count, level1, ncand)
    t.append(time.perf_counter())
    return size, {"local_fallback": 1e3 * (t[-1] - t[0])}


def finalize_from_partials(hist: np.ndarray, sums: np.ndarray, V: np.ndarray, r: np.ndarray, T: np.ndarray,
                           cols: np.ndarray):
    """Host restatement of twosd_cut_finalize (used by the gloo tests): g = sum_v h_v pi_v,
    alpha = g.r + sum_{e RHS} S_e, beta = -T'g - sum_{e T} S_e e_col."""
    h = hist.astype(np.float64) * 2.0 ** -62
    g = h @ V
    alpha = float(g @ r)
    beta = -(T.T @ g)
    for e, c in enumerate(cols):
        if c < 0:
            alpha += sums[1 + e]
        else:
            beta[c] -= sums[1 + e]
    return alpha, beta

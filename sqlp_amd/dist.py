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
    holds the same ordered set (the order decides argmax ties); check_vertex_sets_agree
    compares size + fingerprint across ranks before every cut all-reduce.
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
    """Concatenate every rank's (n_r x m) rows in rank order (variable n_r)."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return rows
    G = dist.get_world_size()
    n = torch.tensor([rows.shape[0]], dtype=torch.int64, device=rows.device)
    counts = [torch.zeros_like(n) for _ in range(G)]
    dist.all_gather(counts, n)
    counts = [int(c.item()) for c in counts]
    mx = max(counts)
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

    def _buffers(self):
        n_u64, n_f64 = self.ctx.cut_partial_len()
        if self.hist is None or self.hist.numel() < n_u64:
            self.hist = torch.zeros(max(n_u64, 1024), dtype=torch.int64, device=self.device)
            self._sync()
        if self.sums is None or self.sums.numel() < n_f64:
            self.sums = torch.zeros(max(n_f64, 256), dtype=torch.float64, device=self.device)
            self._sync()     # torch's fill must land before the library's stream touches the buffer
        return self.hist[:n_u64], self.sums[:n_f64]

    def _sync(self):
        if self.hist is not None and self.hist.is_cuda:
            torch.cuda.synchronize(self.device)

    def build_cut(self, epi, x, total_weight, tie_rel, verify=True):
        """build_sasa_cut over the scenarios of every rank: local partial on this GPU (the
        library zero-fills and writes the buffers on its stream, synchronously), all-reduce,
        identical finalize on every rank.  Returns (alpha, beta)."""
        if verify:
            check_vertex_sets_agree(self.ctx)
        hist, sums = self._buffers()
        self.ctx.cut_partial(epi, x, tie_rel, total_weight, hist.data_ptr(), sums.data_ptr())
        allreduce_cut_partials(hist, sums)
        self._sync()         # the collective runs on torch / RCCL streams, finalize on the library's
        return self.ctx.cut_finalize(x, hist.data_ptr(), sums.data_ptr())


def build_cut_sharded(ctx, epi, x, total_weight, tie_rel, device, verify=True):
    """build_sasa_cut over the scenarios of every rank (one CutExchange per context)."""
    ex = getattr(ctx, "_cut_exchange", None)
    if ex is None:
        ex = ctx._cut_exchange = CutExchange(ctx, device)
    return ex.build_cut(epi, x, total_weight, tie_rel, verify=verify)


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


def refresh_sharded(ctx, train_epi, x, first, count, max_pool, level1=0, ncand=0, device=None):
    """twosd_pool_refresh of the training scenarios of every rank (this rank: [first,
    first + count) of train_epi, the ranks' slices contiguous in rank order) -- the same pool on
    every rank, equal to one rank refreshing from all of them:
      1. each rank solves its slice (twosd_refresh_train);
      2. exchange 1: all-gather of the distinct bases (key, count, first scenario) and of the
         delta boxes; select_refresh_bases on every rank;
      3. each rank composes the picks it owns (twosd_refresh_build_local);
      4. exchange 2: all-gather of the packs (one all_gather_into_tensor of device buffers,
         padded to the largest pack); every rank assembles the pool (twosd_refresh_assemble);
      5. the two-level candidate lists from every rank's picks (exchange 3: the picks).
    Returns (pool size, phase milliseconds)."""
    import time
    rank, G = world()
    t = [time.perf_counter()]
    keys, counts, reps, lo, hi = ctx.refresh_train(train_epi, x, first, count)
    t.append(time.perf_counter())
    if G == 1:
        all_keys, all_counts, all_reps, ns = keys, counts, reps, [len(keys)]
        box_lo, box_hi = lo, hi
    else:
        all_keys, ns = _allgather_1d(keys.view(np.int64), device)
        all_keys = all_keys.view(np.uint64)
        all_counts, _ = _allgather_1d(counts.astype(np.int64), device)
        all_reps, _ = _allgather_1d(reps.astype(np.int64), device)
        boxes, _ = _allgather_1d(np.concatenate([lo, hi]), device)
        boxes = boxes.reshape(G, 2, -1)
        box_lo, box_hi = boxes[:, 0].min(axis=0), boxes[:, 1].max(axis=0)
    rank_of = np.repeat(np.arange(G), ns)
    owner, orep = select_refresh_bases(all_keys, all_counts, all_reps, rank_of, max_pool)
    mine = orep[owner == rank]
    pos = pack_positions(owner, G)
    t.append(time.perf_counter())
    nbytes = ctx.refresh_build_local(mine)
    t.append(time.perf_counter())
    if G == 1:
        buf = torch.empty(nbytes, dtype=torch.uint8, device=device)
        torch.cuda.synchronize(device)
        ctx.refresh_pack(buf.data_ptr())
        size = ctx.refresh_assemble(1, buf.data_ptr(), nbytes, pos, box_lo, box_hi)
    else:
        mx = torch.tensor([nbytes], dtype=torch.int64, device=device if dist.get_backend() == "nccl" else "cpu")
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        stride = (int(mx.item()) + 255) // 256 * 256
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
    t.append(time.perf_counter())
    if level1 > 0 and ncand > 0 and size > level1:
        p1, pf = ctx.pool_candidate_picks(train_epi, x, first, count, level1)
        if G > 1:
            p1, _ = _allgather_1d(p1.astype(np.int64), device)
            pf, _ = _allgather_1d(pf.astype(np.int64), device)
        ctx.pool_set_candidates(level1, ncand, p1, pf)
    t.append(time.perf_counter())
    ms = dict(zip(("train", "select", "build", "exchange_assemble", "candidates"),
                  (1e3 * (b - a) for a, b in zip(t[:-1], t[1:]))))
    return size, ms


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

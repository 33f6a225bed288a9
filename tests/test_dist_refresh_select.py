"""The global basis selection of the distributed pool refresh (sqlp_amd.dist.select_refresh_bases
and its exchange over gloo, world 2 and 3 on CPU): the ranks' per-slice basis lists, merged,
pick the same bases in the same order as one rank listing all training scenarios, which is what
twosd_pool_refresh does (vkey_first_occurrences + stable sort by count, ties by first
occurrence).  No GPU: the per-slice lists are built here from a synthetic stream of basis keys."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from sqlp_amd import dist as sdist


def _stream(T=3000, seed=4):
    """Basis keys of T training scenarios: a Zipf-like mix with many ties in the counts."""
    rng = np.random.default_rng(seed)
    pool = rng.integers(1, 2**63, size=400, dtype=np.int64).astype(np.uint64)
    return pool[np.minimum(rng.zipf(1.3, size=T) - 1, 399)]


def _slice_bases(keys):
    """What twosd_refresh_train lists for one slice: distinct keys in first-occurrence order,
    their counts and first (local) scenario."""
    _, first, inv = np.unique(keys, return_index=True, return_inverse=True)
    order = np.argsort(first)
    cnt = np.bincount(inv)
    return keys[first[order]], cnt[order], first[order]


def _single_rank(keys, max_pool):
    k, c, f = _slice_bases(keys)
    sel = np.argsort(-c, kind="stable")[: max_pool - 1]           # api.hip: stable_sort by count
    return f[sel]


@pytest.mark.parametrize("G", [1, 2, 3, 5])
@pytest.mark.parametrize("max_pool", [2, 17, 64, 1000])
def test_selection_equals_single_rank(G, max_pool):
    keys = _stream()
    T = len(keys)
    parts = [_slice_bases(keys[sdist.shard_range(T, r, G)[0]:sdist.shard_range(T, r, G)[1]]) for r in range(G)]
    kk = np.concatenate([p[0] for p in parts])
    cc = np.concatenate([p[1] for p in parts])
    ff = np.concatenate([p[2] for p in parts])
    rk = np.concatenate([np.full(len(p[0]), r) for r, p in enumerate(parts)])
    owner, rep = sdist.select_refresh_bases(kk, cc, ff, rk, max_pool)
    glob = np.array([sdist.shard_range(T, r, G)[0] for r in owner]) + rep if len(owner) else np.zeros(0)
    np.testing.assert_array_equal(glob, _single_rank(keys, max_pool))
    # every pick belongs to the rank of its key's first occurrence
    for o, g in zip(owner, glob):
        assert sdist.shard_range(T, o, G)[0] <= g < sdist.shard_range(T, o, G)[1]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        keys = _stream()
        lo, hi = sdist.shard_range(len(keys), rank, world)
        k, c, f = _slice_bases(keys[lo:hi])
        # refresh_sharded's exchanges 1 and 2: a fixed header per rank, then one padded row
        hdr = sdist._gather_fixed([len(k), hi - lo, hi - lo])
        ns = [int(v) for v in hdr[:, 0]]
        blo, bhi = np.array([-1.0 - rank, 2.0]), np.array([3.0, 4.0 + rank])   # slice delta boxes
        all_k, all_c, all_f, box_lo, box_hi = sdist.exchange_training_bases(k, c, f, blo, bhi, ns)
        assert box_lo.tolist() == [-world, 2.0] and box_hi.tolist() == [3.0, 3.0 + world]
        owner, rep = sdist.select_refresh_bases(all_k, all_c, all_f, np.repeat(np.arange(world), ns), 64)
        out[rank] = (owner.tolist(), rep.tolist(), ns)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_selection_exchange_gloo(world):
    port = _free_port()
    with mp.get_context("spawn").Manager() as mgr:
        out = mgr.dict()
        mp.start_processes(_worker, args=(world, port, out), nprocs=world, join=True, start_method="spawn")
        res = dict(out)
    keys = _stream()
    T = len(keys)
    ref = _single_rank(keys, 64)
    for r in range(world):
        owner, rep, ns = res[r]
        assert (owner, rep) == (res[0][0], res[0][1])
        glob = [sdist.shard_range(T, o, world)[0] + p for o, p in zip(owner, rep)]
        assert glob == ref.tolist()


class _CapStats:
    """Stand-in for SDContext.refresh_cap_stats: one rank's last large batch."""
    def __init__(self, piv, n):
        self.stats = (piv, n)
        self.refresh_kcap = 0

    def refresh_cap_stats(self):
        return self.stats

    def training_cap(self, ps, pn):
        """The native rule (twosd_training_cap, host code) with no context: setting 0 = auto."""
        import ctypes as C
        from sqlp_amd import _lib
        cap = C.c_int()
        assert _lib.load().twosd_training_cap(None, int(ps), int(pn), C.byref(cap)) == 0
        return cap.value


def _cap_worker(rank, world, port, stats, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    os.environ.pop("TWOSD_TRAIN_KCAP", None)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        out[rank] = sdist.refresh_training_cap(_CapStats(*stats[rank]))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("stats,cap", [([(40960, 4096), (163840, 8192)], 50),     # global mean 16.67
                                       ([(4096, 4096), (0, 0)], 32),              # floor 32
                                       ([(0, 0), (0, 0)], 0)])                     # no batch yet: none
def test_training_cap_is_global(stats, cap):
    """Every rank trains under one cap: 3 x the mean pivots of ALL ranks' last large batches (at
    least 32), whatever each rank's own batch was (per-rank caps broke the pool's
    rank-count independence)."""
    port = _free_port()
    with mp.get_context("spawn").Manager() as mgr:
        out = mgr.dict()
        mp.start_processes(_cap_worker, args=(2, port, stats, out), nprocs=2, join=True, start_method="spawn")
        res = dict(out)
    assert res[0] == res[1] == cap


@pytest.mark.parametrize("max_pool", [1, 2, 5, 64, 5000])
def test_native_selection_equals_numpy(max_pool):
    """twosd_select_refresh_bases (host code of the library, no GPU) against the numpy statement:
    random rank lists with repeated keys across ranks and tied totals."""
    rng = np.random.default_rng(max_pool)
    for G in (1, 3, 8):
        keys = rng.integers(1, 60, size=700, dtype=np.int64).astype(np.uint64)
        counts = rng.integers(1, 4, size=700)
        reps = rng.integers(0, 10000, size=700)
        rank_of = np.sort(rng.integers(0, G, size=700))
        o1, r1 = sdist.select_refresh_bases(keys, counts, reps, rank_of, max_pool)
        o2, r2 = sdist._select_refresh_bases_np(keys, counts, reps, rank_of, max_pool)
        np.testing.assert_array_equal(o1, o2)
        np.testing.assert_array_equal(r1, r2)

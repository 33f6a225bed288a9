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
        all_k, ns = sdist._allgather_1d(k.view(np.int64))
        all_c, _ = sdist._allgather_1d(c.astype(np.int64))
        all_f, _ = sdist._allgather_1d(f.astype(np.int64))
        owner, rep = sdist.select_refresh_bases(all_k.view(np.uint64), all_c, all_f, np.repeat(np.arange(world), ns), 64)
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

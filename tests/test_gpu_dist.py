"""Multi-rank path through the PRODUCT code on one GPU: two ranks on cuda:0 over gloo (the
bench's TWOSD_BENCH_SHARED_GPU rehearsal layout), each with its own context and scenario
shard, running sqlp_amd.dist.build_cut_sharded (real twosd_cut_partial buffers, all-reduce,
twosd_cut_finalize) and push_sharded (exchange 2: local dedup, ordered all-gather, push).
Checked against one rank holding every scenario: the uint64 vertex histogram is
bit-identical, alpha / beta agree to the rounding of the k + 1 fp64 sums, and the merged
vertex set equals a sequential push! of all duals in rank order."""
import os
import socket

import numpy as np
import pytest

from tests import instances as I

pytestmark = pytest.mark.gpu

NAME = "ssn"
N_CUT = 3000
N_PUSH = 96


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _setup():
    from sqlp_amd import smps, twosd
    inst = I.load(NAME)
    ctx = twosd.SDContext(inst["sp2"], inst["sto"])
    x = I.x_ev(NAME)
    ctx.compute_basis(x, smps.mean_values(inst["sto"]))
    V = twosd.sdDualVertexSet(ctx)
    _, _, pis, st = ctx.solve_values(x, I.sample(NAME, 600, 3), want_pi=True)
    V.push_batch(pis[st == 0])
    return ctx, x, V


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from sqlp_amd import dist as sdist
        from sqlp_amd import twosd
        ctx, x, V = _setup()
        vals = I.sample(NAME, N_CUT, 21)
        w = np.random.default_rng(1).uniform(0.5, 1.5, size=N_CUT)
        lo, hi = sdist.shard_range(N_CUT, rank, world)
        epi = twosd.sdEpigraph(ctx, 1.0, 0.0)
        twosd.add_scenarios(epi, vals[lo:hi], w[lo:hi])
        dev = torch.device("cuda", 0)
        a, b = sdist.build_cut_sharded(ctx, epi, x, float(w.sum()), 1e-12, dev)
        hist = ctx._cut_exchange.hist[:ctx.cut_partial_len()[0]].cpu().numpy().copy()
        a2, b2 = sdist.build_cut_sharded(ctx, epi, x, float(w.sum()), 1e-12, dev)   # reused buffers
        # exchange 2: every rank pushes the duals of its own shard of new scenarios
        pv = I.sample(NAME, N_PUSH, 77)
        plo, phi = sdist.shard_range(N_PUSH, rank, world)
        _, _, pis, st = ctx.solve_values(x * 0.97, pv[plo:phi], want_pi=True)
        assert (st == 0).all()
        n = sdist.push_sharded(V, pis)
        out[rank] = dict(a=a, b=b, a2=a2, b2=b2, hist=hist, n=n, V=V.matrix(), fp=V.fingerprint())
    finally:
        dist.destroy_process_group()


def test_two_ranks_on_one_gpu_product_path():
    import torch.multiprocessing as mp
    from sqlp_amd import twosd
    port = _free_port()
    ctxm = mp.get_context("spawn")
    with ctxm.Manager() as mgr:
        out = mgr.dict()
        mp.start_processes(_worker, args=(2, port, out), nprocs=2, join=True, start_method="spawn")
        res = dict(out)
    # one rank holding everything
    import torch
    ctx, x, V = _setup()
    vals = I.sample(NAME, N_CUT, 21)
    w = np.random.default_rng(1).uniform(0.5, 1.5, size=N_CUT)
    epi = twosd.sdEpigraph(ctx, 1.0, 0.0)
    twosd.add_scenarios(epi, vals, w)
    nu, nf = ctx.cut_partial_len()
    dev = torch.device("cuda", 0)
    hist1 = torch.zeros(nu, dtype=torch.int64, device=dev)
    sums1 = torch.zeros(nf, dtype=torch.float64, device=dev)
    torch.cuda.synchronize()
    ctx.cut_partial(epi, x, 1e-12, w.sum(), hist1.data_ptr(), sums1.data_ptr())
    ref = twosd.build_sasa_cut(epi, x, V, tie_rel=1e-12)
    pv = I.sample(NAME, N_PUSH, 77)
    _, _, pis, _ = ctx.solve_values(x * 0.97, pv, want_pi=True)
    V.push_batch(pis)                                  # sequential push! in rank order
    for r in (0, 1):
        o = res[r]
        np.testing.assert_array_equal(o["hist"], hist1.cpu().numpy())
        assert o["a"] == pytest.approx(ref.alpha, rel=1e-12)
        np.testing.assert_allclose(o["b"], ref.beta, rtol=1e-12, atol=1e-12 * (1 + np.abs(ref.beta).max()))
        assert o["a2"] == o["a"] and np.array_equal(o["b2"], o["b"])
        assert o["n"] == len(V)
        np.testing.assert_array_equal(o["V"], V.matrix())
        assert o["fp"] == V.fingerprint()
    assert res[0]["a"] == res[1]["a"]


def test_vertex_set_mismatch_detected():
    """check_vertex_sets_agree raises when the ranks' sets differ (one rank pushed an extra
    vertex), instead of all-reducing histograms of different lengths."""
    import torch.multiprocessing as mp
    port = _free_port()
    with mp.get_context("spawn").Manager() as mgr:
        out = mgr.dict()
        mp.start_processes(_mismatch_worker, args=(2, port, out), nprocs=2, join=True, start_method="spawn")
        res = dict(out)
    assert res[0] == "raised" and res[1] == "raised"


def _mismatch_worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from sqlp_amd import dist as sdist
        ctx, x, V = _setup()
        if rank == 1:
            V.push(np.full(ctx.m, 0.125))
        try:
            sdist.check_vertex_sets_agree(ctx)
            out[rank] = "passed"
        except RuntimeError:
            out[rank] = "raised"
    finally:
        dist.destroy_process_group()


# ---- distributed pool refresh (sqlp_amd.dist.refresh_sharded) ------------------------------
R_TRAIN = 4096
R_POOL = 512
R_EVAL = 3000


def _refresh_x():
    from tests.test_gpu_pool_refresh import _sd_x
    return _sd_x(3)


def _storm_ctx():
    from sqlp_amd import smps, twosd
    inst = I.load("storm")
    ctx = twosd.SDContext(inst["sp2"], inst["sto"])
    ctx.compute_basis(I.x_ev("storm"), smps.mean_values(inst["sto"]))
    ctx.set_distributions(inst["sto"])
    return ctx


def _pool_state(ctx, x):
    from sqlp_amd import twosd
    heads = np.stack([ctx.pool_get(p) for p in range(ctx.pool_size())])
    ev = twosd.sdEpigraph(ctx, 1.0, 0.0)
    twosd.add_sampled_scenarios(ev, R_EVAL, 99)
    obj, _, _, st = twosd.solve_batch(ev, x, 0, R_EVAL, want_pi=False)
    return heads, obj, st, ctx.last_pool_picks(R_EVAL), ctx.lp_stats()[0]


def _refresh_worker(rank, world, port, x, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from sqlp_amd import dist as sdist
        from sqlp_amd import twosd
        ctx = _storm_ctx()
        lo, hi = sdist.shard_range(R_TRAIN, rank, world)
        tr = twosd.sdEpigraph(ctx, 1.0, 0.0)
        twosd.add_sampled_scenarios(tr, hi - lo, 4242, first_index=lo)
        size, ms = sdist.refresh_sharded(ctx, tr, x, 0, hi - lo, R_POOL, 128, 160, torch.device("cuda", 0))
        heads, obj, st, picks, piv = _pool_state(ctx, x)
        out[rank] = dict(size=size, heads=heads, obj=obj, st=st, picks=picks, piv=piv, ms=ms)
    finally:
        dist.destroy_process_group()


def test_refresh_sharded_equals_single_rank():
    """Two ranks on cuda:0 (gloo) refresh the pool from their halves of the training scenarios
    (train, exchange the distinct bases, compose the owned picks, all-gather the packs,
    assemble, candidate lists from both ranks' picks): both hold the pool one rank builds from
    all training scenarios with twosd_pool_refresh + twosd_pool_build_candidates -- the same
    bases in the same order -- and the next solve is bit-identical (objectives, pool picks,
    pivots)."""
    import torch.multiprocessing as mp
    from sqlp_amd import twosd
    x = _refresh_x()
    port = _free_port()
    with mp.get_context("spawn").Manager() as mgr:
        out = mgr.dict()
        mp.start_processes(_refresh_worker, args=(2, port, x, out), nprocs=2, join=True, start_method="spawn")
        res = dict(out)
    ctx = _storm_ctx()
    tr = twosd.sdEpigraph(ctx, 1.0, 0.0)
    twosd.add_sampled_scenarios(tr, R_TRAIN, 4242)
    size = ctx.pool_refresh(tr, x, 0, R_TRAIN, R_POOL)
    ctx.pool_build_candidates(tr, x, 0, R_TRAIN, 128, 160)
    heads, obj, st, picks, piv = _pool_state(ctx, x)
    assert size > 128 and (st == 0).all()
    for r in (0, 1):
        o = res[r]
        assert o["size"] == size
        np.testing.assert_array_equal(o["heads"], heads)
        np.testing.assert_array_equal(o["st"], st)
        np.testing.assert_array_equal(o["obj"], obj)
        np.testing.assert_array_equal(o["picks"], picks)
        assert o["piv"] == piv
    print(f"refresh_sharded: pool {size}, phases (rank 0) {res[0]['ms']}")


def _refresh_worker_capped(rank, world, port, x, out):
    """As _refresh_worker, but each rank first solves a batch of >= 4096 scenarios of its own
    size (4096 + 2048 rank), so the ranks' last-batch pivot means differ."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    os.environ.pop("TWOSD_TRAIN_KCAP", None)
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from sqlp_amd import dist as sdist
        from sqlp_amd import twosd
        ctx = _storm_ctx()
        warm = twosd.sdEpigraph(ctx, 1.0, 0.0)
        nw = 4096 + 2048 * rank
        twosd.add_sampled_scenarios(warm, nw, 777, first_index=100000 * rank)
        twosd.solve_batch(warm, I.x_ev("storm"), 0, nw, want_pi=False)
        lo, hi = sdist.shard_range(R_TRAIN, rank, world)
        tr = twosd.sdEpigraph(ctx, 1.0, 0.0)
        twosd.add_sampled_scenarios(tr, hi - lo, 4242, first_index=lo)
        size, ms = sdist.refresh_sharded(ctx, tr, x, 0, hi - lo, R_POOL, 128, 160, torch.device("cuda", 0))
        heads, obj, st, picks, piv = _pool_state(ctx, x)
        out[rank] = dict(size=size, heads=heads, obj=obj, st=st, picks=picks, piv=piv, kcap=ms["kcap"],
                         own=ctx.refresh_cap_stats())
    finally:
        dist.destroy_process_group()


def test_refresh_sharded_capped_equals_single_rank():
    """After batches of different sizes on the two ranks, both train under ONE cap (3 x the mean
    pivots over both ranks' batches) and hold the pool a single rank builds under that cap."""
    import math
    import torch.multiprocessing as mp
    from sqlp_amd import twosd
    x = _refresh_x()
    port = _free_port()
    with mp.get_context("spawn").Manager() as mgr:
        out = mgr.dict()
        mp.start_processes(_refresh_worker_capped, args=(2, port, x, out), nprocs=2, join=True, start_method="spawn")
        res = dict(out)
    (s0, n0), (s1, n1) = res[0]["own"], res[1]["own"]
    assert (n0, n1) == (4096, 6144)
    cap = max(32, math.ceil(3.0 * (s0 + s1) / (n0 + n1)))
    assert res[0]["kcap"] == res[1]["kcap"] == cap
    ctx = _storm_ctx()
    ctx.set_refresh_kcap(cap)
    tr = twosd.sdEpigraph(ctx, 1.0, 0.0)
    twosd.add_sampled_scenarios(tr, R_TRAIN, 4242)
    size = ctx.pool_refresh(tr, x, 0, R_TRAIN, R_POOL)
    ctx.pool_build_candidates(tr, x, 0, R_TRAIN, 128, 160)
    heads, obj, st, picks, piv = _pool_state(ctx, x)
    for r in (0, 1):
        o = res[r]
        assert o["size"] == size
        np.testing.assert_array_equal(o["heads"], heads)
        np.testing.assert_array_equal(o["obj"], obj)
        np.testing.assert_array_equal(o["picks"], picks)
        assert o["piv"] == piv
    print(f"capped refresh_sharded: cap {cap}, pool {size}")


def test_refresh_sharded_g1_auto_cap_equals_pool_refresh(monkeypatch):
    """One rank, the auto training cap (no setting, no TWOSD_TRAIN_KCAP): refresh_sharded derives
    the cap through the native rule (twosd_training_cap) from the same last-batch statistics
    twosd_pool_refresh reads, so both build the same pool (the Python copy of the rule
    differed at an exact-integer 3 x mean and for TWOSD_TRAIN_KCAP=0)."""
    import math
    from sqlp_amd import dist as sdist
    from sqlp_amd import twosd
    monkeypatch.delenv("TWOSD_TRAIN_KCAP", raising=False)
    x = _refresh_x()
    states, caps = [], []
    for sharded in (True, False):
        ctx = _storm_ctx()
        warm = twosd.sdEpigraph(ctx, 1.0, 0.0)
        twosd.add_sampled_scenarios(warm, 6144, 777)
        twosd.solve_batch(warm, I.x_ev("storm"), 0, 6144, want_pi=False)
        ps, pn = ctx.refresh_cap_stats()
        assert pn == 6144
        cap = ctx.training_cap(ps, pn)
        assert cap == max(32, math.ceil(3 * ps / pn))
        assert ctx.training_cap(ps, 0) == 0                 # no large batch yet: no cap
        tr = twosd.sdEpigraph(ctx, 1.0, 0.0)
        twosd.add_sampled_scenarios(tr, R_TRAIN, 4242)
        if sharded:
            import torch
            size, ms = sdist.refresh_sharded(ctx, tr, x, 0, R_TRAIN, R_POOL, 128, 160, torch.device("cuda", 0))
            caps.append(ms["kcap"])
        else:
            size = ctx.pool_refresh(tr, x, 0, R_TRAIN, R_POOL)
            ctx.pool_build_candidates(tr, x, 0, R_TRAIN, 128, 160)
            caps.append(cap)
        states.append((size,) + _pool_state(ctx, x))
    assert caps[0] == caps[1]
    (s0, h0, o0, st0, p0, v0), (s1, h1, o1, st1, p1, v1) = states
    assert s0 == s1
    np.testing.assert_array_equal(h0, h1)
    np.testing.assert_array_equal(o0, o1)
    np.testing.assert_array_equal(p0, p1)
    assert v0 == v1


def test_training_cap_setting_and_env(monkeypatch):
    """twosd_training_cap: an explicit setting wins, a negative one means no cap, and
    TWOSD_TRAIN_KCAP is read as a setting (0 = auto) on the native side for every caller."""
    ctx = _storm_ctx()
    monkeypatch.delenv("TWOSD_TRAIN_KCAP", raising=False)
    assert ctx.training_cap(11 * 1000, 1000) == 33              # 3 x the mean, an exact integer: no round-up
    assert ctx.training_cap(100, 1000) == 32                    # floor 32
    ctx.set_refresh_kcap(40)
    assert ctx.training_cap(100, 1000) == 40
    ctx.set_refresh_kcap(-1)
    assert ctx.training_cap(100000, 1000) == 0
    ctx.set_refresh_kcap(0)
    monkeypatch.setenv("TWOSD_TRAIN_KCAP", "0")
    assert ctx.training_cap(50000, 1000) == 150
    monkeypatch.setenv("TWOSD_TRAIN_KCAP", "77")
    assert ctx.training_cap(50000, 1000) == 77

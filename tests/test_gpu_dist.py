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

"""GPU dual-vertex-set dedup (push!, dual_set.jl:84-94) vs the oracle's linear scan."""
import numpy as np
import pytest

from oracle import twosd_ref
from tests import instances as I

pytestmark = pytest.mark.gpu


def _ctx(name):
    from sqlp_amd import twosd
    inst = I.load(name)
    return twosd.SDContext(inst["sp2"], inst["sto"])


def test_dual_set_kat_on_device():
    # test/dual_set_test.jl with the length-3 vectors (newsvendor has m2 = 3)
    from sqlp_amd import twosd
    ctx = _ctx("newsvendor")
    V = twosd.sdDualVertexSet(ctx)
    sizes = []
    for v in ([1., 2, 3], [1.0000000001, 2, 3], [4., 5, 6], [3., 2, 1]):
        twosd.push(V, np.array(v))
        sizes.append(len(V))
    assert sizes == [1, 1, 2, 3]
    with pytest.raises(ValueError):          # length mismatch: the device set has fixed m2
        V.push(np.array([4., 5, 6, 7]))
    V.clear()
    assert len(V) == 0
    idx = twosd.sdDualVertexSet(ctx).push_batch(np.array([[1., 2, 3], [1.0000000001, 2, 3], [4., 5, 6], [4., 5, 6],
                                                           [3., 2, 1], [-0.0, 1, 1], [0.0, 1, 1]]))
    assert idx.tolist() == [0, 0, 1, 1, 2, 3, 3]     # -0.0 == 0.0 in Julia's r1 != r2


def _candidates(m, rng, nbase=60, n=400):
    base = np.round(rng.normal(size=(nbase, m)) * rng.choice([1, 10, 1000], size=(nbase, 1)), 4)
    base[rng.random(size=base.shape) < 0.6] = 0.0
    picks = rng.integers(0, nbase, size=n)
    C = base[picks].copy()
    kind = rng.integers(0, 5, size=n)
    C[kind == 1] *= 1 + 1e-12                            # rounding-equal (almost always)
    C[kind == 2] += rng.normal(size=(np.sum(kind == 2), m)) * 1e-3   # different
    C[kind == 3, 0] = -C[kind == 3, 0]                   # sign flip of one component
    C[kind == 4] = C[kind == 4] * (1 + 2.0 ** -15)       # right at the 16-bit granularity
    return C


@pytest.mark.parametrize("name", ["ssn", "transship"])
def test_push_batches_match_linear_scan(name):
    ctx = _ctx(name)
    from sqlp_amd import twosd
    rng = np.random.default_rng(11)
    C = _candidates(ctx.m, rng)
    V = twosd.sdDualVertexSet(ctx)
    ref = twosd_ref.DualVertexSet()
    for blk in np.array_split(C, [1, 50, 51, 220]):      # batches of 1, 49, 1, 169, 180
        got = V.push_batch(blk)
        want = [ref.push(v) for v in blk]
        assert got.tolist() == want
    assert len(V) == len(ref)
    np.testing.assert_array_equal(V.matrix(), ref.matrix(ctx.m))


def test_nan_vectors_always_appended():
    from sqlp_amd import twosd
    ctx = _ctx("newsvendor")
    V = twosd.sdDualVertexSet(ctx)
    idx = V.push_batch(np.array([[np.nan, 1, 1], [np.nan, 1, 1], [1.0, 1, 1], [1.0, 1, 1]]))
    assert idx.tolist() == [0, 1, 2, 2]


def test_truncate_rebuilds_lookup():
    from sqlp_amd import twosd
    ctx = _ctx("transship")
    rng = np.random.default_rng(2)
    C = np.round(rng.normal(size=(30, ctx.m)), 3)
    V = twosd.sdDualVertexSet(ctx)
    V.push_batch(C)
    V.truncate(10)
    idx = V.push_batch(C)
    assert idx[:10].tolist() == list(range(10)) and idx[10:].tolist() == list(range(10, 30))

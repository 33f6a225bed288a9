"""The vectorised oracle push (twosd_ref.DualVertexSet.push_batch, used as the checker of large
GPU pushes) against the line-by-line restatement of push! (dual_set.jl:84-94): the same vertex
set in the same order and the same index for every pushed vector; round16_vec against round16
on edge values (zeros, subnormals, the overflow guard, halfway cases, non-finite)."""
import numpy as np

from oracle import twosd_ref as T


def test_round16_vec_equals_round16():
    rng = np.random.default_rng(0)
    x = np.concatenate([rng.normal(size=2000) * 10.0 ** rng.integers(-300, 300, 2000),
                        [0.0, -0.0, np.inf, -np.inf, np.nan, 5e-324, 2.0 ** -1010, 2.0 ** -1008, 2.0 ** -1007,
                         1.7976931348623157e308, -1.7976931348623157e308, 0.5 + 2.0 ** -17, 1.5 * 2.0 ** -17,
                         -3.0 * 2.0 ** -17, 1 + 2.0 ** -16, 1 + 3 * 2.0 ** -16]])
    a = T.round16_vec(x)
    b = np.array([T.round16(v) for v in x])
    assert np.array_equal(a.view(np.uint64), b.view(np.uint64))


def test_push_batch_equals_sequential_push():
    rng = np.random.default_rng(1)
    base = rng.normal(size=(40, 12)) * 100
    rows = []
    for _ in range(600):
        v = base[rng.integers(0, 40)].copy()
        u = rng.random()
        if u < 0.2:
            v[rng.integers(0, 12)] *= 1 + 2.0 ** -50       # equal after round16
        elif u < 0.3:
            v[rng.integers(0, 12)] *= 1 + 2.0 ** -10       # a new vertex
        elif u < 0.32:
            v[rng.integers(0, 12)] = np.nan                # never equal to anything
        rows.append(v)
    P = np.array(rows)
    seq = T.DualVertexSet()
    idx_seq = [seq.push(v) for v in P]
    fast = T.DualVertexSet()
    idx_fast = np.concatenate([fast.push_batch(P[:250]), fast.push_batch(P[250:])])
    assert idx_fast.tolist() == idx_seq
    assert len(fast) == len(seq)
    assert np.array_equal(fast.matrix(), seq.matrix(), equal_nan=True)
    assert fast.hashes == seq.hashes
    # a batch push onto a set built by single pushes
    mixed = T.DualVertexSet(list(P[:100]))
    assert mixed.push_batch(P[100:]).tolist() == idx_seq[100:]

"""ctypes wrapper for oracle/cpu_lp.c (TEST INFRASTRUCTURE ONLY -- see oracle/__init__.py).

``CpuLP`` is the CPU restatement of the per-scenario LP solve (solve_problem!,
src/smps/smps_routines.jl:50-62) and ``build_cut`` the reference-order
argmax_procedure + build_sasa_cut (subprob.jl:141-169, epigraph.jl:125-146).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "liboracle_cpu.so")
_lib = None

ST_OPTIMAL, ST_INFEASIBLE, ST_ITER_LIMIT, ST_NUMERIC = 0, 1, 2, 3


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = C.CDLL(_LIB_PATH)
        P = C.c_void_p
        L.oracle_lp_create.restype = P
        L.oracle_lp_create.argtypes = [C.c_int, C.c_int, P, P, P, P, P]
        L.oracle_lp_destroy.argtypes = [P]
        L.oracle_lp_set_basis.argtypes = [P, P]
        L.oracle_lp_basis_dual_infeas.argtypes = [P]
        L.oracle_lp_basis_dual_infeas.restype = C.c_double
        L.oracle_lp_solve_from_slack.argtypes = [P, P, P, P, P]
        L.oracle_lp_solve_batch.argtypes = [P, C.c_int, C.c_int, P, P, P, C.c_int, P, P, P, P, P, C.c_int]
        L.oracle_lp_set_pool.argtypes = [P, C.c_int, P]
        L.oracle_lp_solve_batch_pool.argtypes = [P, C.c_int, C.c_int, P, P, P, C.c_int, P, P, P, P, P, C.c_int]
        L.oracle_build_cut.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, P, P, P, P, P, P, P,
                                       C.c_double, P, P, P, P, C.c_int]
        L.oracle_dense_inverse.argtypes = [C.c_int, P, P]
        L.oracle_philox4x32_10.argtypes = [P, P, P]
        L.oracle_sample.argtypes = [C.c_int, C.c_int, C.c_uint64, C.c_uint64, P, P, P, P, P, P, P, P]
        _lib = L
    return _lib


def _p(a):
    return a.ctypes.data_as(C.c_void_p) if a is not None else None


def dense_to_csc(W):
    W = np.asarray(W, dtype=np.float64)
    m, n = W.shape
    colptr = [0]
    rows, vals = [], []
    for j in range(n):
        nz = np.nonzero(W[:, j])[0]
        rows.extend(nz.tolist())
        vals.extend(W[nz, j].tolist())
        colptr.append(len(rows))
    return (np.array(colptr, dtype=np.int32), np.array(rows, dtype=np.int32),
            np.array(vals, dtype=np.float64))


class CpuLP:
    """Warm-started dual simplex on min q'y, W y (senses) b, y >= 0."""

    def __init__(self, W, q, senses):
        self.m, self.n = W.shape
        self.colptr, self.rowidx, self.val = dense_to_csc(W)
        self.q = np.ascontiguousarray(q, dtype=np.float64)
        self.sense = np.frombuffer("".join(senses).encode(), dtype=np.int8).copy()
        self.h = lib().oracle_lp_create(self.m, self.n, _p(self.colptr), _p(self.rowidx), _p(self.val),
                                        _p(self.q), _p(self.sense))
        self.head0 = None

    def __del__(self):
        if getattr(self, "h", None) and _lib is not None:
            _lib.oracle_lp_destroy(self.h)
            self.h = None

    def solve_from_slack(self, b):
        b = np.ascontiguousarray(b, dtype=np.float64)
        head = np.zeros(self.m, dtype=np.int32)
        obj = C.c_double(); it = C.c_int()
        st = lib().oracle_lp_solve_from_slack(self.h, _p(b), _p(head), C.byref(obj), C.byref(it))
        return st, obj.value, head, it.value

    def set_basis(self, head0):
        self.head0 = np.ascontiguousarray(head0, dtype=np.int32)
        rc = lib().oracle_lp_set_basis(self.h, _p(self.head0))
        if rc != 0:
            raise RuntimeError("singular basis")
        return lib().oracle_lp_basis_dual_infeas(self.h)

    def solve_batch(self, rows, base, DR, kmax=512, want_y=False, nthreads=0):
        DR = np.ascontiguousarray(DR, dtype=np.float64)
        N, k = DR.shape
        rows = np.ascontiguousarray(rows, dtype=np.int32)
        base = np.ascontiguousarray(base, dtype=np.float64)
        obj = np.zeros(N); pi = np.zeros((N, self.m)); st = np.zeros(N, dtype=np.int32)
        it = np.zeros(N, dtype=np.int32)
        y = np.zeros((N, self.n)) if want_y else None
        lib().oracle_lp_solve_batch(self.h, N, k, _p(rows), _p(base), _p(DR), kmax, _p(obj), _p(pi),
                                    _p(y), _p(st), _p(it), nthreads)
        return obj, pi, y, st, it


    def set_pool(self, heads):
        """Warm-start pool: P bases (P x m heads) with dense inverses (setup)."""
        self.pool_heads = np.ascontiguousarray(heads, dtype=np.int32)
        rc = lib().oracle_lp_set_pool(self.h, self.pool_heads.shape[0], _p(self.pool_heads))
        if rc != 0:
            raise RuntimeError(f"singular pool basis {-1 - rc}")

    def solve_batch_pool(self, rows, base, DR, kmax=512, nthreads=0):
        """solve_batch with each scenario started from the pool basis of least total primal
        infeasibility (the GPU's level-1 selection key); returns obj, pi, st, iters, picks."""
        DR = np.ascontiguousarray(DR, dtype=np.float64)
        N, k = DR.shape
        rows = np.ascontiguousarray(rows, dtype=np.int32)
        base = np.ascontiguousarray(base, dtype=np.float64)
        obj = np.zeros(N); pi = np.zeros((N, self.m)); st = np.zeros(N, dtype=np.int32)
        it = np.zeros(N, dtype=np.int32); picks = np.zeros(N, dtype=np.int32)
        lib().oracle_lp_solve_batch_pool(self.h, N, k, _p(rows), _p(base), _p(DR), kmax, _p(obj), _p(pi),
                                         _p(st), _p(it), _p(picks), nthreads)
        return obj, pi, st, it, picks


def build_cut(r, T, x, V, rows, DR, w, tie_rel=0.0, nthreads=0):
    r = np.ascontiguousarray(r, dtype=np.float64)
    T = np.ascontiguousarray(T, dtype=np.float64)
    x = np.ascontiguousarray(x, dtype=np.float64)
    V = np.ascontiguousarray(V, dtype=np.float64)
    DR = np.ascontiguousarray(DR, dtype=np.float64)
    w = np.ascontiguousarray(w, dtype=np.float64)
    rows = np.ascontiguousarray(rows, dtype=np.int32)
    m, n1 = T.shape
    N, k = DR.shape
    nv = V.shape[0]
    alpha = C.c_double()
    beta = np.zeros(n1)
    mv = np.zeros(N); ma = np.zeros(N, dtype=np.int32)
    lib().oracle_build_cut(m, n1, nv, N, k, _p(rows), _p(r), _p(T), _p(x), _p(V), _p(DR), _p(w),
                           float(tie_rel), C.byref(alpha), _p(beta), _p(mv), _p(ma), nthreads)
    return alpha.value, beta, mv, ma


def philox4x32_10(ctr, key):
    """Philox4x32-10 block (published algorithm, restated in oracle/sampler.c)."""
    c = np.ascontiguousarray(ctr, dtype=np.uint32)
    k = np.ascontiguousarray(key, dtype=np.uint32)
    out = np.zeros(4, dtype=np.uint32)
    lib().oracle_philox4x32_10(_p(c), _p(k), _p(out))
    return out


def sample_deltas(sto, positions, template_values, N, seed, first_index=0):
    """N x k scenario deltas (value - template) of the device sampler's stream."""
    kinds, off, vals, probs, p0, p1 = [], [0], [], [], [], []
    for pos in positions:
        d = sto.indep[pos]
        if d[0] == "DISCRETE":
            order = np.argsort(np.asarray(d[1]), kind="stable")
            kinds.append(0); vals += list(np.asarray(d[1])[order]); probs += list(np.asarray(d[2])[order])
            p0.append(0.0); p1.append(0.0)
        elif d[0] == "NORMAL":
            kinds.append(1); p0.append(d[1]); p1.append(float(np.sqrt(d[2])))
        else:
            kinds.append(2); p0.append(d[1]); p1.append(d[2])
        off.append(len(vals))
    k = len(positions)
    a = [np.ascontiguousarray(kinds, dtype=np.int32), np.ascontiguousarray(off, dtype=np.int32),
         np.ascontiguousarray(vals if vals else [0.0]), np.ascontiguousarray(probs if probs else [0.0]),
         np.ascontiguousarray(p0, dtype=np.float64), np.ascontiguousarray(p1, dtype=np.float64),
         np.ascontiguousarray(template_values, dtype=np.float64)]
    out = np.zeros((N, k))
    lib().oracle_sample(int(N), k, C.c_uint64(seed), C.c_uint64(first_index), *[_p(v) for v in a], _p(out))
    return out

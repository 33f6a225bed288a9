"""TwoSD hot-path restatement (oracle; TEST INFRASTRUCTURE ONLY -- see oracle/__init__.py).

Pure-numpy restatement of the reference's Julia, in the reference's loop order:
  * ``round16``             <- Julia ``round(x; base=2, sigdigits=16)`` as used at
                               src/sd_algorithm/dual_set.jl:32-33,51 (Base._round_sigdigits)
  * ``hash_dual_vector``    <- dual_set.jl:46-53
  * ``dual_isequal``        <- dual_set.jl:24-40
  * ``DualVertexSet.push``  <- dual_set.jl:84-94 (linear scan, first occurrence kept)
  * ``Coefficients``        <- subprob.jl:4-12 / extract_coefficients subprob.jl:15-69
  * ``delta_coefficients``  <- subprob.jl:104-121
  * ``eval_dual``           <- subprob.jl:128-131
  * ``argmax_procedure``    <- subprob.jl:141-169
  * ``build_sasa_cut``      <- epigraph.jl:125-146
  * ``add_cut_discount`` / ``evaluate_epigraph`` <- epigraph.jl:101-117, 177-203
  * ``remove_cuts_by_multiplier`` <- algorithm.jl:57-72 (CUT_REMOVE_TOLERANCE algorithm.jl:23)
  * ``sync_cuts``           <- cell.jl:139-201 (remove_cuts! + add_cut_to_master! per epigraph)
  * ``evaluate_multi_epigraph`` / ``check_improvement`` <- epigraph.jl:221-228, improvement.jl:19-49
"""
from __future__ import annotations

import math
import struct
import numpy as np

SIGNIFICANT_DIGITS = 16          # dual_set.jl:4


def round16(x: float) -> float:
    """Julia round(x; base=2, sigdigits=16): digits = 16 - (1 + exponent(x)); scale by
    an exact power of two, round half-to-even, scale back.  Returns x itself when the
    scale overflows (Julia's _round_digits non-finite guard)."""
    x = float(x)
    if x == 0.0 or not math.isfinite(x):     # Base.round: `isfinite(x) || return x`
        return x
    m, e2 = math.frexp(x)           # x = m * 2**e2, 0.5 <= |m| < 1  -> exponent(x) = e2-1
    digits = SIGNIFICANT_DIGITS - e2
    try:
        if digits >= 0:
            sc = 2.0 ** digits
            r = round(x * sc) / sc
        else:
            isc = 2.0 ** (-digits)
            r = round(x / isc) * isc
    except OverflowError:
        return x
    if not math.isfinite(r):
        return x
    return float(r)


def round16_array(v) -> np.ndarray:
    return np.array([round16(t) for t in np.asarray(v, dtype=np.float64)], dtype=np.float64)


def round16_vec(a) -> np.ndarray:
    """round16 elementwise, vectorised (the same values as round16 on every element): the scale
    by 2**digits is exact, np.round rounds half to even like Python's round, and the cases where
    round16 returns x itself -- 0, non-finite, a scale 2**digits that overflows (digits > 1023),
    a non-finite result -- keep x."""
    x = np.asarray(a, dtype=np.float64)
    out = x.copy()
    fin = np.isfinite(x) & (x != 0.0)
    _, e2 = np.frexp(np.where(fin, x, 1.0))
    digits = SIGNIFICANT_DIGITS - e2
    pos = fin & (digits >= 0) & (digits <= 1023)
    neg = fin & (digits < 0)
    with np.errstate(over="ignore", invalid="ignore"):
        rp = np.round(np.ldexp(np.where(pos, x, 0.0), np.where(pos, digits, 0))) / np.ldexp(1.0, np.where(pos, digits, 0))
        isc = np.ldexp(1.0, np.where(neg, -digits, 0))
        rn = np.round(np.where(neg, x, 0.0) / isc) * isc
    r = np.where(pos, rp, np.where(neg, rn, x))
    ok = (pos | neg) & np.isfinite(r)
    out[ok] = r[ok]
    return out


def hash_dual_vector(vec) -> int:
    s = 0.0
    for v in np.asarray(vec, dtype=np.float64):   # sequential sum, dual_set.jl:47-50
        s += abs(float(v))
    return struct.unpack("<Q", struct.pack("<d", round16(s)))[0]


def dual_isequal(h1, d1, h2, d2) -> bool:
    if len(d1) != len(d2) or h1 != h2:
        return False
    for a, b in zip(d1, d2):
        if round16(a) != round16(b):
            return False
    return True


class DualVertexSet:
    """sdDualVertexSet: insertion-ordered unique vertices (dual_set.jl:69-127)."""

    def __init__(self, data=None):
        self.hashes: list[int] = []
        self.data: list[np.ndarray] = []
        if data is not None:
            for d in data:
                self.push(d)

    def push(self, vec) -> int:
        """Returns the index of the (existing or new) vertex equal to vec."""
        vec = np.asarray(vec, dtype=np.float64)
        h = hash_dual_vector(vec)
        for i, (hv, dv) in enumerate(zip(self.hashes, self.data)):
            if dual_isequal(h, vec, hv, dv):
                return i
        self.hashes.append(h)
        self.data.append(vec)
        return len(self.data) - 1

    def push_batch(self, pis) -> np.ndarray:
        """push! of every row of pis in order (dual_set.jl:84-94), vectorised for large batches:
        the same hashes (sequential L1 sum, round16) and the same equality test (equal hash, then
        every component equal after round16), with the linear scan restricted to the vertices of
        equal hash -- dual_isequal is false for any other, so the first match in insertion order
        is the same.  Returns the vertex index of every row."""
        P = np.atleast_2d(np.asarray(pis, dtype=np.float64))
        if not hasattr(self, "_by_hash"):
            self._by_hash = {}
            self._r16 = []
            for i, (h, d) in enumerate(zip(self.hashes, self.data)):
                self._by_hash.setdefault(h, []).append(i)
                self._r16.append(round16_vec(d))
        sums = np.cumsum(np.abs(P), axis=1)[:, -1] if P.shape[1] else np.zeros(P.shape[0])
        hb = round16_vec(sums).view(np.uint64)
        R = round16_vec(P)
        out = np.empty(P.shape[0], dtype=np.int64)
        for s in range(P.shape[0]):
            h = int(hb[s])
            hit = -1
            for i in self._by_hash.get(h, ()):
                if len(self.data[i]) == P.shape[1] and np.array_equal(self._r16[i], R[s]):
                    hit = i
                    break
            if hit < 0:
                hit = len(self.data)
                self.hashes.append(h)
                self.data.append(P[s].copy())
                self._r16.append(R[s])
                self._by_hash.setdefault(h, []).append(hit)
            out[s] = hit
        return out

    def __len__(self):
        return len(self.data)

    def __iter__(self):
        return iter(self.data)

    def matrix(self, m=None) -> np.ndarray:
        if not self.data:
            return np.zeros((0, m or 0))
        return np.vstack(self.data)


class Coefficients:
    """sdSubprobCoefficients (subprob.jl:4-12): r, T, W + name lookups."""

    def __init__(self, sp):
        self.rhs = sp.r.copy()
        self.transfer = sp.T.copy()
        self.recourse = sp.W.copy()
        self.col_lookup = {n: i for i, n in enumerate(sp.last_names)}
        self.row_lookup = {n: i for i, n in enumerate(sp.row_names)}


def delta_coefficients(coef: Coefficients, scenario):
    """subprob.jl:104-121.  scenario = [((col_name,row_name), value), ...].
    Raises KeyError for unknown rows/columns exactly like the Dict lookups."""
    dr = np.zeros(len(coef.rhs))
    dT = np.zeros(coef.transfer.shape)
    for (col, row), val in scenario:
        i = coef.row_lookup[row]
        if col == "RHS" or col == "rhs":
            dr[i] = val - coef.rhs[i]
        else:
            j = coef.col_lookup[col]
            dT[i, j] = val - coef.transfer[i, j]
    return dr, dT


def eval_dual(coef: Coefficients, delta, x, dual) -> float:
    dr, dT = delta
    return float(np.dot(dual, (coef.rhs + dr) - (coef.transfer + dT) @ x))


def tie_tolerance(M: float, rel: float) -> float:
    return rel * (1.0 + abs(M))


def _seq_base(coef: Coefficients, x):
    """r - (T x) as the reference writes it (`coef.rhs - coef.transfer * x`, subprob.jl:147):
    T x accumulated from zero column by column (SparseArrays' CSC mat-vec, tx[i] += T[i, j] x[j]
    for j ascending; a structural zero adds an exact 0), then subtracted from r; each product
    and sum rounded on its own (oracle_build_cut's arithmetic)."""
    prod = coef.transfer * x[None, :]
    tx = np.zeros(prod.shape[0])
    for j in range(prod.shape[1]):
        tx = tx + prod[:, j]
    return np.array(coef.rhs, dtype=np.float64) - tx


def _seq_rowdot(A, b):
    """sum_i A[v, i] b[i] for every row v, in index order (np.cumsum adds sequentially; the
    products are rounded first: no contraction)."""
    if A.shape[1] == 0:
        return np.zeros(A.shape[0])
    return np.cumsum(A * b[None, :], axis=1)[:, -1]


def _element_terms(dr, dT, x):
    """(row, coef_e * dv_e) of every nonzero random element of a scenario, by ascending row (RHS
    element first, then T columns ascending): the terms restated_score adds one at a time."""
    rows, fac = [], []
    dT = np.asarray(dT)
    for i in np.flatnonzero((np.asarray(dr) != 0) | (dT != 0).any(axis=1)):
        if dr[i] != 0:
            rows.append(i)
            fac.append(float(dr[i]))
        for j in np.flatnonzero(dT[i]):
            rows.append(i)
            fac.append(float(-x[j]) * float(dT[i, j]))
    return np.array(rows, dtype=np.int64), np.array(fac, dtype=np.float64)


def argmax_procedure(coef: Coefficients, deltas, x, V, tie_rel: float = 0.0):
    """subprob.jl:141-169 (MIN_SENSE).  tie_rel == 0 is the reference rule exactly (strict
    '>' so the first maximum in insertion order wins).  tie_rel > 0 is the build's
    documented near-tie rule: the lowest vertex index whose score is within
    tie_rel*(1+|max|) of the maximum.
    Scores s = dot(pi, r - T x) + dot(pi, dvec) (:147-155) with both dots sequential and no
    contraction -- oracle_build_cut's arithmetic, which the GPU's decisions are pinned to: the
    base dot in row order, the delta dot over the random elements by ascending row, one term
    pi[row] * (coef_e * dv_e) per element (coef_e = 1 for an RHS element, -x[col] for a T
    element; within a row the RHS element first, then T columns ascending).  With one random
    element per row this is the dense dot(pi, dvec) with its zero rows dropped (adding an exact
    0 changes nothing).  The reference's OpenBLAS ddot adds in a CPU-dependent blocked order, so
    at rounding-level ties its pick is not reproducible by any restatement."""
    x = np.asarray(x, dtype=np.float64)
    base = _seq_base(coef, x)
    Vl = list(V)
    vals, args = [], []
    Vm = np.array(Vl, dtype=np.float64).reshape(len(Vl), -1)
    vb = _seq_rowdot(Vm, base)
    for dr, dT in deltas:
        rows, fac = _element_terms(dr, dT, x)
        t = _seq_rowdot(Vm[:, rows], fac) if len(rows) else np.zeros(len(Vl))
        scores = [float(s) for s in (vb + t)]
        if tie_rel == 0.0:
            best, arg = -math.inf, -1
            for i, s in enumerate(scores):
                if s > best:
                    best, arg = s, i
        else:
            M = max(scores)
            tol = tie_tolerance(M, tie_rel)
            arg = next(i for i, s in enumerate(scores) if s >= M - tol)
            best = scores[arg]
        vals.append(best)
        args.append(arg)
    return np.array(vals), np.array(args, dtype=np.int64)


def build_sasa_cut(coef: Coefficients, deltas, weights, x, V, tie_rel: float = 0.0):
    """epigraph.jl:125-146.  Returns (alpha, beta, weight_mark, max_val, max_arg)."""
    max_val, max_arg = argmax_procedure(coef, deltas, x, V, tie_rel)
    Vl = list(V)
    total = float(sum(weights))           # epi.total_scenario_weight (epigraph.jl:89)
    alpha = 0.0
    beta = np.zeros(len(x))
    for i, (dr, dT) in enumerate(deltas):
        dual = Vl[max_arg[i]]
        p = weights[i] / total
        alpha += p * float(np.dot(dual, coef.rhs + dr))
        beta += -p * ((coef.transfer + dT).T @ dual)
    return alpha, beta, total, max_val, max_arg


def add_cut_discount(alpha, beta, discount, lower_bound):
    """epigraph.jl:105-106 (the rhs/coefficients add_cut_to_master! writes)."""
    return discount * alpha + (1 - discount) * lower_bound, discount * np.asarray(beta)


CUT_REMOVE_TOLERANCE = 0.001      # algorithm.jl:23


def remove_cuts_by_multiplier(cuts, duals, tol=CUT_REMOVE_TOLERANCE):
    """algorithm.jl:57-72 for one epigraph: duals[j] is dual(cell.epicon_ref[i][j]); every j
    with |dual| < tol is collected into delete_index, then deleteat!(epi.cuts, delete_index)."""
    delete_index = []
    for j in range(len(duals)):
        if abs(duals[j]) < tol:
            delete_index.append(j)
    return [c for j, c in enumerate(cuts) if j not in delete_index]


def sync_cuts(epis):
    """cell.jl:198-201 -> :167-192 for every epigraph in order: its rows are removed, then each
    cut is added with discount = weight_mark / total_scenario_weight (add_cut_to_master!,
    epigraph.jl:101-117), then the incumbent cut with discount 1.  epis = [(cuts,
    incumbent_cut, total_scenario_weight, lower_bound)], cuts = [(alpha, beta, weight_mark)].
    Returns the master's epigraph rows in insertion order: (epi, alpha', beta', incumbent)."""
    rows = []
    for e, (cuts, inc, tw, lb) in enumerate(epis):
        for a, b, wm in cuts:
            na, nb = add_cut_discount(a, b, wm / tw, lb)
            rows.append((e, na, nb, False))
        if inc is not None:
            na, nb = add_cut_discount(inc[0], inc[1], 1.0, lb)
            rows.append((e, na, nb, True))
    return rows


def evaluate_epigraph(cuts, incumbent_cut, x, total_scenario_weight, lower_bound):
    """epigraph.jl:177-203 (MIN_SENSE).  cuts = [(alpha, beta, weight_mark)]."""
    best = lower_bound
    for a, b, wm in cuts:
        d = wm / total_scenario_weight
        v = d * (a + float(np.dot(b, x))) + (1 - d) * lower_bound
        if v > best:
            best = v
    if incumbent_cut is not None:
        a, b, _ = incumbent_cut
        v = a + float(np.dot(b, x))
        if v > best:
            best = v
    return best


INCUMBENT_SELECTION_Q = 0.2        # improvement.jl:1


def evaluate_multi_epigraph(infos, x):
    """epigraph.jl:221-228 over (objective_weight, cuts, incumbent_cut, total_weight,
    lower_bound) tuples; cuts = [(alpha, beta, weight_mark)]."""
    return sum(w * evaluate_epigraph(cuts, inc, x, tw, lb) for w, cuts, inc, tw, lb in infos)


def check_improvement(f_last, f_current, x_candidate, x_incumbent, f_cand, f_inc):
    """improvement.jl:19-49 (MIN_SENSE): returns (candidate_estimation, incumbent_estimation,
    required_improvement, is_improved)."""
    ce = evaluate_multi_epigraph(f_current, x_candidate) + f_cand
    ie = evaluate_multi_epigraph(f_current, x_incumbent) + f_inc
    lce = evaluate_multi_epigraph(f_last, x_candidate) + f_cand
    lie = evaluate_multi_epigraph(f_last, x_incumbent) + f_inc
    req_impr = INCUMBENT_SELECTION_Q * (lce - lie)
    return ce, ie, req_impr, ce < ie + req_impr

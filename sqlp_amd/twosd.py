"""Host-side mirror of the reference's TwoSD hot-path API, backed by libtwosd_hip.so.

Reference (module TwoSD, yhz0/SQLP) -> here:
  sdDualVertexSet / push!         dual_set.jl:69-127      -> sdDualVertexSet / push / .push
  sdEpigraph(prob, w, lb)         epigraph.jl:52-61       -> sdEpigraph(ctx, w, lb)
  add_scenario!(epi, w, weight)   epigraph.jl:81-96       -> add_scenario / add_scenarios
  solve_problem!(sp, x, w)        smps_routines.jl:50-62  -> solve_problem / solve_batch
  evaluate(sp1, sp2, sto, x; N)   smps_routines.jl:67-82  -> evaluate
  argmax_procedure(...)           subprob.jl:141-169      -> argmax_procedure
  build_sasa_cut(epi, x, V)       epigraph.jl:125-146     -> build_sasa_cut -> sdCut
  sd_iteration! (hot segment)     algorithm.jl:45-55,79-85 -> sd_iteration_hot_path
All arithmetic runs on the GPU through the C ABI; there is no CPU fallback.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field

import numpy as np

from . import _lib
from ._lib import check, ptr
from .smps import spStageProblem, spSmpsPosition, scenario_positions

MIN_SENSE = "MIN_SENSE"
# argmax tie rule: 0 = the reference's strict '>' (subprob.jl:156, first maximum in insertion
# order).  tie_rel > 0 is the build's near-tie rule (lowest vertex index within
# tie_rel * (1 + |max|) of the maximum), which makes the pick independent of summation order
# for scores that tie in exact arithmetic; the bench passes 1e-12 explicitly.
DEFAULT_TIE_REL = 0.0


def _f64(a):
    return np.ascontiguousarray(a, dtype=np.float64)


@dataclass
class sdCut:
    """eta >= alpha + beta'x (epigraph.jl:5-12); never scaled."""
    alpha: float
    beta: np.ndarray
    weight_mark: float


class SDContext:
    """Device-resident hot-path state of one cell on one GPU: the stage-2 template
    (extract_coefficients, subprob.jl:15-69), the random-element layout, the shared
    warm-start basis, and the dual vertex set (cell.dual_vertices, cell.jl:25)."""

    def __init__(self, sp2: spStageProblem, sto=None, positions=None, device: int = 0, index_base: int = 0):
        """index_base = 1 hands the template and positions to the library 1-based, as a Julia
        caller passes SparseMatrixCSC colptr / rowval (twosd_set_template, index_base)."""
        self.lib = _lib.load()
        self.index_base = int(index_base)
        h = C.c_void_p()
        check(self.lib.twosd_create(device, C.byref(h)))
        self.h = h
        self.sp2 = sp2
        self.m, self.n1, self.n2 = sp2.shape
        Tcp, Trv, Tnz = sp2.T
        Wcp, Wrv, Wnz = sp2.W
        ib = self.index_base
        self._keep = [np.ascontiguousarray(a + ib if a.dtype.kind == "i" else a)
                      for a in (Tcp, Trv, Tnz, Wcp, Wrv, Wnz)]
        sense = np.frombuffer("".join(sp2.sense).encode(), dtype=np.int8).copy()
        self._keep += [sense]
        check(self.lib.twosd_set_template(
            self.h, self.m, self.n1, self.n2,
            ptr(self._keep[0]), ptr(self._keep[1]), ptr(self._keep[2]),
            ptr(self._keep[3]), ptr(self._keep[4]), ptr(self._keep[5]),
            ptr(_f64(sp2.q)), ptr(_f64(sp2.r)), ptr(sense), ptr(_f64(sp2.ylb)), ptr(_f64(sp2.yub)), ib))
        self.row_lookup = {n: i for i, n in enumerate(sp2.stage_constraints)}
        self.col_lookup = {n: j for j, n in enumerate(sp2.last_stage_vars)}
        if sto is not None and positions is None:
            positions = list(sto.indep.keys())
        self.set_positions(positions or [])
        self.has_basis = False

    def set_positions(self, positions):
        """Random-element layout; KeyError for an unknown row/column like
        delta_coefficients (subprob.jl:112,116)."""
        self.positions = [spSmpsPosition(*p) for p in positions]
        self.pos_index = {p: e for e, p in enumerate(self.positions)}
        rows = np.array([self.row_lookup[p.row_name] for p in self.positions], dtype=np.int32)
        cols = np.array([-1 if p.col_name in ("RHS", "rhs") else self.col_lookup[p.col_name]
                         for p in self.positions], dtype=np.int32)
        self.k = len(self.positions)
        self.rows, self.cols = rows, cols
        ib = self.index_base
        rows_b = np.ascontiguousarray(rows + ib, dtype=np.int32)
        cols_b = np.ascontiguousarray(np.where(cols < 0, -1, cols + ib), dtype=np.int32)
        check(self.lib.twosd_set_random_positions(self.h, self.k, ptr(rows_b), ptr(cols_b), ib))
        # template value of every element (for scenario -> values conversion)
        T = self.sp2.dense_T()
        self.template_values = np.array(
            [self.sp2.r[r] if c < 0 else T[r, c] for r, c in zip(rows, cols)], dtype=np.float64)

    def close(self):
        if getattr(self, "h", None):
            self.lib.twosd_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -- warm-start basis -------------------------------------------------------
    def compute_basis(self, x, values=None):
        """Optimal basis of the scenario `values` (default: template) at x, installed as the
        shared warm start of every scenario solve."""
        x = _f64(x)
        v = None if values is None else _f64(values)
        check(self.lib.twosd_compute_basis(self.h, ptr(x), ptr(v)))
        self.has_basis = True

    def set_basis(self, head):
        head = np.ascontiguousarray(head, dtype=np.int32)
        check(self.lib.twosd_set_basis(self.h, ptr(head)))
        self.has_basis = True

    def get_basis(self):
        head = np.zeros(self.m, dtype=np.int32)
        check(self.lib.twosd_get_basis(self.h, ptr(head)))
        return head

    # -- warm-start basis pool (twosd_pool_*: fewer pivots, identical vertices) ---
    def pool_add_basis(self, head) -> bool:
        head = np.ascontiguousarray(head, dtype=np.int32)
        added = C.c_int(0)
        check(self.lib.twosd_pool_add_basis(self.h, ptr(head), C.byref(added)))
        return bool(added.value)

    def pool_build(self, epi, x, first, count, max_pool) -> int:
        """Add the most frequent optimal bases of scenarios [first, first+count) of `epi`
        at x to the pool (up to max_pool bases); returns the pool size."""
        x = _f64(x)
        n = C.c_int(0)
        check(self.lib.twosd_pool_build(self.h, epi.index, ptr(x), int(first), int(count), int(max_pool),
                                        C.byref(n)))
        return n.value

    def pool_build_candidates(self, epi, x, first, count, level1, ncand):
        """Two-level warm-start selection: level 1 over the first `level1` pool bases, level 2
        over the `ncand` bases a flat selection picks most often for the training scenarios
        [first, first+count) of `epi` that share the level-1 pick.  level1 = 0: flat."""
        check(self.lib.twosd_pool_build_candidates(self.h, epi.index, ptr(_f64(x)), int(first), int(count),
                                                   int(level1), int(ncand)))

    def last_pool_picks(self, N):
        """Pool basis every scenario of the last LP batch started from."""
        picks = np.zeros(N, dtype=np.int32)
        check(self.lib.twosd_last_pool_picks(self.h, int(N), ptr(picks)))
        return picks

    def invalidate_x(self):
        """Drop the per-x cache (next solve / cut recomputes it; results unchanged)."""
        check(self.lib.twosd_invalidate_x(self.h))

    def pool_refresh(self, epi, x, first, count, max_pool) -> int:
        """Replace the warm-start pool by the primary basis plus the max_pool - 1 most frequent
        optimal bases of training scenarios [first, first+count) of epi at x (twosd_pool_refresh)."""
        n = C.c_int()
        check(self.lib.twosd_pool_refresh(self.h, epi.index, ptr(_f64(x)), first, count, max_pool, C.byref(n)))
        return n.value

    # -- distributed refresh (twosd_refresh_*; driven by sqlp_amd.dist.refresh_sharded) --------
    def refresh_train(self, epi, x, first, count):
        """Training solves of this rank's slice; returns (keys u64, counts, first scenarios, box
        lo, box hi) of its distinct optimal bases."""
        U = C.c_int()
        lo = np.zeros(max(self.k, 1))
        hi = np.zeros(max(self.k, 1))
        check(self.lib.twosd_refresh_train(self.h, epi.index, ptr(_f64(x)), int(first), int(count), C.byref(U),
                                           ptr(lo), ptr(hi)))
        keys = np.zeros(U.value, dtype=np.uint64)
        counts = np.zeros(U.value, dtype=np.int32)
        reps = np.zeros(U.value, dtype=np.int32)
        check(self.lib.twosd_refresh_train_bases(self.h, ptr(keys), ptr(counts), ptr(reps)))
        return keys, counts, reps, lo[:self.k], hi[:self.k]

    def refresh_train_ex(self, epi, x, first, count, kcap):
        """Training solves of this rank's slice under the pivot cap kcap (> 0; <= 0 none), one
        launch, no retry (twosd_refresh_train_ex); returns (keys u64, counts, first scenarios,
        box lo, box hi, optimal training scenarios)."""
        U = C.c_int()
        nopt = C.c_int()
        lo = np.zeros(max(self.k, 1))
        hi = np.zeros(max(self.k, 1))
        check(self.lib.twosd_refresh_train_ex(self.h, epi.index, ptr(_f64(x)), int(first), int(count), int(kcap),
                                              C.byref(U), C.byref(nopt), ptr(lo), ptr(hi)))
        keys = np.zeros(U.value, dtype=np.uint64)
        counts = np.zeros(U.value, dtype=np.int32)
        reps = np.zeros(U.value, dtype=np.int32)
        check(self.lib.twosd_refresh_train_bases(self.h, ptr(keys), ptr(counts), ptr(reps)))
        return keys, counts, reps, lo[:self.k], hi[:self.k], nopt.value

    def refresh_cap_stats(self):
        """(pivot sum, scenarios) of the last LP batch of >= 4096 scenarios: the scale of the
        training pivot cap (twosd_refresh_cap_stats)."""
        s = C.c_int64()
        n = C.c_int64()
        check(self.lib.twosd_refresh_cap_stats(self.h, C.byref(s), C.byref(n)))
        return s.value, n.value

    def cut_stats(self):
        """(scenarios re-decided in the restatement's arithmetic, candidates scored, full
        re-scans, dominated twin vertices left out) of the last cut (twosd_cut_stats)."""
        out = np.zeros(4, dtype=np.int64)
        check(self.lib.twosd_cut_stats(self.h, ptr(out)))
        return tuple(int(v) for v in out)

    def cut_pass(self):
        """(fp32, band) of the last cut: 1 if its MFMA pass ran in fp32, 0 for fp64, and that
        pass's decision band (twosd_cut_pass)."""
        f = C.c_int()
        b = C.c_double()
        check(self.lib.twosd_cut_pass(self.h, C.byref(f), C.byref(b)))
        return f.value, b.value

    def training_cap(self, pivots_sum, scenarios) -> int:
        """The refresh's training pivot cap for a last large batch of `scenarios` solves with
        `pivots_sum` pivots (twosd_training_cap: the native rule, this context's setting)."""
        cap = C.c_int()
        check(self.lib.twosd_training_cap(self.h, int(pivots_sum), int(scenarios), C.byref(cap)))
        return cap.value

    def last_objective(self):
        """(sum_s w_s obj_s, sum_s w_s) of the last solve_batch / solve_push / solve_values batch
        (twosd_last_objective): the incumbent objective at x is their quotient."""
        a = C.c_double()
        b = C.c_double()
        check(self.lib.twosd_last_objective(self.h, C.byref(a), C.byref(b)))
        return a.value, b.value

    def refresh_build_local(self, reps) -> int:
        """Compose the bases this rank owns (first scenarios `reps`, selection order); returns the
        pack size in bytes."""
        reps = np.ascontiguousarray(reps, dtype=np.int32)
        nb = C.c_int64()
        check(self.lib.twosd_refresh_build_local(self.h, len(reps), ptr(reps), C.byref(nb)))
        return nb.value

    def refresh_pack(self, d_dst: int):
        check(self.lib.twosd_refresh_pack(self.h, C.c_void_p(d_dst)))

    def refresh_assemble(self, G, d_packs: int, stride: int, order, box_lo, box_hi) -> int:
        order = np.ascontiguousarray(order, dtype=np.int32)
        n = C.c_int()
        check(self.lib.twosd_refresh_assemble(self.h, int(G), C.c_void_p(d_packs), C.c_int64(stride), len(order),
                                              ptr(order), ptr(_f64(box_lo)), ptr(_f64(box_hi)), C.byref(n)))
        return n.value

    def pool_candidate_picks(self, epi, x, first, count, level1):
        p1 = np.zeros(count, dtype=np.int32)
        pf = np.zeros(count, dtype=np.int32)
        check(self.lib.twosd_pool_candidate_picks(self.h, epi.index, ptr(_f64(x)), int(first), int(count), int(level1),
                                                  ptr(p1), ptr(pf)))
        return p1, pf

    def pool_set_candidates(self, level1, ncand, p1, pf):
        p1 = np.ascontiguousarray(p1, dtype=np.int32)
        pf = np.ascontiguousarray(pf, dtype=np.int32)
        check(self.lib.twosd_pool_set_candidates(self.h, int(level1), int(ncand), len(p1), ptr(p1), ptr(pf)))

    def set_refresh_kcap(self, kcap: int):
        """Pivot cap of the refresh's training solves: > 0 explicit, 0 auto (3 x the mean pivots of
        the last batch of >= 4096 scenarios, at least 32), < 0 none (the kernel's kmax)."""
        check(self.lib.twosd_set_refresh_kcap(self.h, int(kcap)))
        self.refresh_kcap = int(kcap)

    def last_lp_iters(self, N):
        """(pivots, status) of the first N scenarios of the last LP launch."""
        it = np.zeros(N, dtype=np.int32)
        st = np.zeros(N, dtype=np.int32)
        check(self.lib.twosd_last_lp_iters(self.h, int(N), ptr(it), ptr(st)))
        return it, st

    def last_refresh_ms(self):
        """[training solves, re-solves, host composition, upload, total] of the last refresh."""
        out = np.zeros(5)
        check(self.lib.twosd_last_refresh_ms(self.h, ptr(out)))
        return out

    def pool_size(self) -> int:
        n = C.c_int(0)
        check(self.lib.twosd_pool_size(self.h, C.byref(n)))
        return n.value

    def pool_get(self, p):
        head = np.zeros(self.m, dtype=np.int32)
        check(self.lib.twosd_pool_get(self.h, int(p), ptr(head)))
        return head

    # -- on-device scenario sampler (rand(rng, sto), smps_sto.jl:117-149) ----------
    def set_distributions(self, sto):
        """Upload the independent distribution of every random element (position order)."""
        kinds, nsup, vals, probs, p0, p1 = [], [], [], [], [], []
        for pos in self.positions:
            d = sto.indep[pos]
            if d[0] == "DISCRETE":
                kinds.append(0); nsup.append(len(d[1])); vals += list(d[1]); probs += list(d[2])
                p0.append(0.0); p1.append(0.0)
            elif d[0] == "NORMAL":
                kinds.append(1); nsup.append(0); p0.append(d[1]); p1.append(d[2])
            else:
                kinds.append(2); nsup.append(0); p0.append(d[1]); p1.append(d[2])
        a = [np.ascontiguousarray(kinds, dtype=np.int32), np.ascontiguousarray(nsup, dtype=np.int32),
             _f64(vals if vals else [0.0]), _f64(probs if probs else [0.0]), _f64(p0), _f64(p1)]
        check(self.lib.twosd_set_distributions(self.h, self.k, *[ptr(v) for v in a]))

    def scenario_values(self, scenario) -> np.ndarray:
        """spSmpsScenario (list of position => value) -> value vector in layout order.
        Elements a scenario omits keep their template value (delta 0)."""
        v = self.template_values.copy()
        for pos, val in scenario:
            pos = spSmpsPosition(*pos)
            if pos not in self.pos_index:
                # unknown position: KeyError on its row / column like subprob.jl:112,116
                self.row_lookup[pos.row_name]
                if pos.col_name not in ("RHS", "rhs"):
                    self.col_lookup[pos.col_name]
                raise KeyError(f"{pos} is not a random element of this context")
            v[self.pos_index[pos]] = val
        return v

    def timings_us(self):
        """[LP kernel, dedup, cut partial, cut finalize, pool selection] of the last calls."""
        t = np.zeros(5)
        check(self.lib.twosd_last_timings(self.h, ptr(t)))
        return t

    def lp_stats(self):
        s = C.c_int64()
        mx = C.c_int()
        check(self.lib.twosd_last_lp_stats(self.h, C.byref(s), C.byref(mx)))
        return s.value, mx.value

    def lp_eta_entries(self) -> int:
        """Eta-arena entries (12 B each) the last LP batch wrote (twosd_last_lp_eta_entries)."""
        return self.lp_counts()[0]

    def lp_counts(self):
        """(eta-arena entries, pool starts retried from the primary basis) of the last LP batch."""
        e = C.c_int64()
        r = C.c_int64()
        check(self.lib.twosd_last_lp_eta_entries(self.h, C.byref(e), C.byref(r)))
        return e.value, r.value

    def last_push_reps(self) -> int:
        """Scenarios whose dual the last solve_push recovered and pushed (first scenario of
        each distinct optimal dual vertex of the batch)."""
        r = C.c_int()
        check(self.lib.twosd_last_push_reps(self.h, C.byref(r)))
        return r.value

    def last_push_mode(self) -> int:
        """1 if the last solve_push recovered every dual in its main pass (full mode), 0 if it
        re-solved the representatives (twosd_last_push_mode)."""
        r = C.c_int()
        check(self.lib.twosd_last_push_mode(self.h, C.byref(r)))
        return r.value

    def lp_flops(self):
        """Counted fp64 FLOPs of the last LP batch (2 * row width per executed row op)."""
        ops = C.c_int64()
        w = C.c_int()
        check(self.lib.twosd_last_lp_ops(self.h, C.byref(ops), C.byref(w)))
        return 2.0 * w.value * ops.value

    # -- multi-GPU split of build_sasa_cut (device buffers from the caller) --------
    def cut_partial_len(self):
        a = C.c_int64()
        b = C.c_int64()
        check(self.lib.twosd_cut_partial_len(self.h, C.byref(a), C.byref(b)))
        return a.value, b.value

    def cut_partial(self, epi, x, tie_rel, total_weight, d_hist_ptr, d_sums_ptr):
        check(self.lib.twosd_cut_partial(self.h, epi.index, ptr(_f64(x)), float(tie_rel), float(total_weight),
                                         C.c_void_p(d_hist_ptr), C.c_void_p(d_sums_ptr), None, None))

    def cut_finalize(self, x, d_hist_ptr, d_sums_ptr):
        a = C.c_double()
        beta = np.zeros(self.n1)
        check(self.lib.twosd_cut_finalize(self.h, ptr(_f64(x)), C.c_void_p(d_hist_ptr), C.c_void_p(d_sums_ptr),
                                          C.byref(a), ptr(beta)))
        return a.value, beta

    # -- solve_problem! / evaluate ----------------------------------------------
    def solve_values(self, x, values, want_pi=True, want_y=False, raise_on_status=True):
        values = _f64(np.atleast_2d(values))
        N = values.shape[0]
        obj = np.zeros(N)
        st = np.zeros(N, dtype=np.int32)
        pi = np.zeros((N, self.m)) if want_pi else None
        y = np.zeros((N, self.n2)) if want_y else None
        rc = self.lib.twosd_solve_values(self.h, ptr(_f64(x)), N, ptr(values), ptr(obj), ptr(pi), ptr(y), ptr(st))
        if rc != 0 and not (rc == -4 and not raise_on_status):
            check(rc)
        return obj, y, pi, st


class sdDualVertexSet:
    """Device-resident dual vertex set of an SDContext (dual_set.jl:69-127).  There is one
    set per context (the cell's shared set)."""

    def __init__(self, ctx: SDContext, data=None):
        self.ctx = ctx
        if data is not None:
            self.push_batch(np.atleast_2d(np.asarray(data, dtype=np.float64)))

    def push(self, vec):
        """push!(dvs, vec): appends iff no equal vertex exists; returns self (dual_set.jl:84-94)."""
        self.push_batch(np.asarray(vec, dtype=np.float64)[None, :])
        return self

    def push_batch(self, pis) -> np.ndarray:
        """Sequential push! of every row; returns the vertex index of each row."""
        pis = _f64(np.atleast_2d(pis))
        if pis.shape[1] != self.ctx.m:
            raise ValueError(f"dual vector length {pis.shape[1]} != {self.ctx.m}")
        out = np.zeros(pis.shape[0], dtype=np.int32)
        ns = C.c_int()
        check(self.ctx.lib.twosd_dvs_push(self.ctx.h, pis.shape[0], ptr(pis), ptr(out), C.byref(ns)))
        return out

    def __len__(self):
        s = C.c_int()
        check(self.ctx.lib.twosd_dvs_size(self.ctx.h, C.byref(s)))
        return s.value

    def matrix(self, first=0, count=None) -> np.ndarray:
        n = len(self)
        count = n - first if count is None else count
        out = np.zeros((count, self.ctx.m))
        check(self.ctx.lib.twosd_dvs_get(self.ctx.h, first, count, ptr(out)))
        return out

    def __iter__(self):
        return iter(list(self.matrix()))

    def clear(self):
        check(self.ctx.lib.twosd_dvs_clear(self.ctx.h))

    def truncate(self, size):
        check(self.ctx.lib.twosd_dvs_truncate(self.ctx.h, int(size)))

    def fingerprint(self) -> int:
        """Order-dependent 64-bit digest of the set (twosd_dvs_fingerprint)."""
        d = C.c_uint64()
        check(self.ctx.lib.twosd_dvs_fingerprint(self.ctx.h, C.byref(d)))
        return d.value


def push(dvs: sdDualVertexSet, vec):
    return dvs.push(vec)


class sdEpigraph:
    """sdEpigraph (epigraph.jl:17-61): scenario pool + weights on the device, cuts on the host."""

    def __init__(self, ctx: SDContext, objective_weight: float, lower_bound: float):
        self.ctx = ctx
        self.objective_weight = float(objective_weight)
        self.lower_bound = float(lower_bound)
        e = C.c_int()
        check(ctx.lib.twosd_epigraph_create(ctx.h, C.byref(e)))
        self.index = e.value
        self.scenario_weight: list = []
        self.cuts: list = []
        self.incumbent_cut = None

    @property
    def total_scenario_weight(self) -> float:
        tw = C.c_double()
        check(self.ctx.lib.twosd_epigraph_info(self.ctx.h, self.index, None, C.byref(tw)))
        return tw.value

    @property
    def num_scenarios(self) -> int:
        n = C.c_int()
        check(self.ctx.lib.twosd_epigraph_info(self.ctx.h, self.index, C.byref(n), None))
        return n.value


def add_scenario(epi: sdEpigraph, scenario, weight: float = 1.0):
    """add_scenario!(epi, scenario, weight) (epigraph.jl:81-96)."""
    add_scenarios(epi, epi.ctx.scenario_values(scenario)[None, :], np.array([weight]))


def add_scenarios(epi: sdEpigraph, values, weights=None):
    """Batched add_scenario!: values N x k (layout order), weights N (default 1.0)."""
    values = _f64(np.atleast_2d(values))
    N = values.shape[0]
    w = None if weights is None else _f64(weights)
    check(epi.ctx.lib.twosd_add_scenarios(epi.ctx.h, epi.index, N, ptr(values), ptr(w)))
    epi.scenario_weight.extend([1.0] * N if w is None else list(w))


def add_sampled_scenarios(epi: sdEpigraph, N, seed, first_index=0, weights=None):
    """N scenarios drawn on the device (Philox4x32-10 stream (seed, first_index + s, e))
    appended to epi -- add_scenario!(epi, rand(rng, sto)) N times without a host copy."""
    w = None if weights is None else _f64(weights)
    check(epi.ctx.lib.twosd_add_sampled_scenarios(epi.ctx.h, epi.index, int(N), C.c_uint64(seed),
                                                   C.c_uint64(first_index), ptr(w)))
    epi.scenario_weight.extend([1.0] * N if w is None else list(w))


def get_scenarios(epi: sdEpigraph, first=0, count=None) -> np.ndarray:
    """Element values (template + stored delta) of scenarios [first, first+count)."""
    if count is None:
        count = epi.num_scenarios - first
    out = np.zeros((count, epi.ctx.k))
    check(epi.ctx.lib.twosd_get_scenarios(epi.ctx.h, epi.index, int(first), int(count), ptr(out)))
    return out


def solve_batch(epi: sdEpigraph, x, first=0, count=None, want_pi=True, want_y=False):
    """solve_problem! over scenarios [first, first+count) of epi at x -> (obj, y, pi, status)."""
    ctx = epi.ctx
    count = epi.num_scenarios - first if count is None else count
    obj = np.zeros(count)
    st = np.zeros(count, dtype=np.int32)
    pi = np.zeros((count, ctx.m)) if want_pi else None
    y = np.zeros((count, ctx.n2)) if want_y else None
    check(ctx.lib.twosd_solve_batch(ctx.h, epi.index, ptr(_f64(x)), first, count, ptr(obj), ptr(pi), ptr(y), ptr(st)))
    return obj, y, pi, st


def solve_problem(ctx: SDContext, x, scenario):
    """solve_problem!(sp, x, scenario) -> (obj, y_opt, dual_opt) (smps_routines.jl:50-62).
    A non-optimal LP raises (the reference logs @error and returns junk duals)."""
    obj, y, pi, st = ctx.solve_values(x, ctx.scenario_values(scenario)[None, :], want_pi=True, want_y=True)
    return float(obj[0]), y[0], pi[0]


def evaluate(ctx: SDContext, first_stage_cost, x, values):
    """evaluate(sp1, sp2, sto, x; N) (smps_routines.jl:67-82) on given sampled values:
    c'x + (1/N) sum_w obj_w.  first_stage_cost: the stage-1 objective vector."""
    obj, _, _, _ = ctx.solve_values(x, values, want_pi=False)
    N = obj.shape[0]
    s2 = 0.0
    for o in obj:                      # s2_cost += 1/N*obj, in sample order (:79)
        s2 += 1.0 / N * o
    return float(np.dot(first_stage_cost, x)) + s2


def evaluate_sampled(ctx: SDContext, first_stage_cost, x, N, seed, first=0, count=None):
    """evaluate(sp1, sp2, sto, x; N) (smps_routines.jl:67-82) with the N scenarios drawn on
    the device (needs ctx.set_distributions): c'x + sum_w (1/N) obj_w in scenario order.
    first/count select a shard of the stream (the c'x term is added by every caller of
    a shard; multi-GPU: sqlp_amd.dist.evaluate_sharded)."""
    count = N - first if count is None else count
    s2 = C.c_double()
    check(ctx.lib.twosd_evaluate_sampled(ctx.h, ptr(_f64(x)), C.c_int64(N), C.c_int64(first), C.c_int64(count),
                                         C.c_uint64(seed), C.byref(s2)))
    return float(np.dot(first_stage_cost, x)) + s2.value


def evaluate_epigraph(cuts, incumbent_cut, x, total_scenario_weight, lower_bound, sense=MIN_SENSE):
    """Pointwise max (MIN sense) of the discounted cuts and the incumbent cut at x, floored by
    the lower bound; no epigraph weight (epigraph.jl:177-203)."""
    best = lower_bound
    x = np.asarray(x, dtype=np.float64)
    for cut in cuts:
        discount = cut.weight_mark / total_scenario_weight
        val = discount * (cut.alpha + float(np.dot(cut.beta, x))) + (1 - discount) * lower_bound
        if (sense == MIN_SENSE and val > best) or (sense != MIN_SENSE and val < best):
            best = val
    if incumbent_cut is not None:
        val = incumbent_cut.alpha + float(np.dot(incumbent_cut.beta, x))
        if (sense == MIN_SENSE and val > best) or (sense != MIN_SENSE and val < best):
            best = val
    return best


def evaluate_epigraph_weighted(epi: sdEpigraph, x, sense=MIN_SENSE):
    """objective_weight * evaluate_epigraph over the epigraph's cuts (epigraph.jl:205-219)."""
    return epi.objective_weight * evaluate_epigraph(epi.cuts, epi.incumbent_cut, x, epi.total_scenario_weight,
                                                    epi.lower_bound, sense=sense)


def evaluate_multi_epigraph(epis, x, sense=MIN_SENSE):
    """Sum of the weighted epigraph values (epigraph.jl:221-228)."""
    return sum(evaluate_epigraph_weighted(e, x, sense=sense) for e in epis)


INCUMBENT_SELECTION_Q = 0.2


@dataclass
class sdImprovementInfo:
    candidate_estimation: float
    incumbent_estimation: float
    required_improvement: float
    is_improved: bool


def check_improvement(f_last, f_current, f_cand, f_inc, x_candidate, x_incumbent, sense=MIN_SENSE):
    """Incumbent selection (improvement.jl:19-49).  f_cand / f_inc are the values of the
    common (first-stage) expression at the candidate / incumbent (evaluate_expr)."""
    ce = evaluate_multi_epigraph(f_current, x_candidate, sense) + f_cand
    ie = evaluate_multi_epigraph(f_current, x_incumbent, sense) + f_inc
    lce = evaluate_multi_epigraph(f_last, x_candidate, sense) + f_cand
    lie = evaluate_multi_epigraph(f_last, x_incumbent, sense) + f_inc
    req_impr = INCUMBENT_SELECTION_Q * (lce - lie)
    req = ie + req_impr
    improved = ce < req if sense == MIN_SENSE else ce > req
    return sdImprovementInfo(ce, ie, req_impr, improved)


def argmax_procedure(epi: sdEpigraph, x, dual_vertices: sdDualVertexSet, tie_rel=DEFAULT_TIE_REL):
    """(max_val, max_arg) over every scenario of epi (subprob.jl:141-169); max_arg holds
    0-based vertex indices into dual_vertices (the reference returns Refs to vectors)."""
    cut, mv, ma = _build_cut(epi, x, tie_rel, want_argmax=True)
    return mv, ma


def build_sasa_cut(epi: sdEpigraph, x, dual_vertices: sdDualVertexSet, tie_rel=DEFAULT_TIE_REL) -> sdCut:
    """build_sasa_cut(epi, x, V) (epigraph.jl:125-146)."""
    cut, _, _ = _build_cut(epi, x, tie_rel, want_argmax=False)
    return cut


def _build_cut(epi, x, tie_rel, want_argmax):
    ctx = epi.ctx
    a = C.c_double()
    wm = C.c_double()
    beta = np.zeros(ctx.n1)
    N = epi.num_scenarios
    mv = np.zeros(N) if want_argmax else None
    ma = np.zeros(N, dtype=np.int32) if want_argmax else None
    check(ctx.lib.twosd_build_cut(ctx.h, epi.index, ptr(_f64(x)), float(tie_rel), C.byref(a), ptr(beta),
                                  C.byref(wm), ptr(mv), ptr(ma)))
    return sdCut(a.value, beta, wm.value), mv, ma


def solve_push(epi: sdEpigraph, x, first, count, want_obj=True):
    """Device-side solve_problem! + push! of the duals (no host round trip).  want_obj=False
    skips the copy of the objectives and statuses (sd_iteration! does not read them; a
    non-optimal scenario still raises); obj and st are then None."""
    ctx = epi.ctx
    obj = np.zeros(count) if want_obj else None
    st = np.zeros(count, dtype=np.int32) if want_obj else None
    ns = C.c_int()
    check(ctx.lib.twosd_solve_push(ctx.h, epi.index, ptr(_f64(x)), first, count, ptr(obj) if want_obj else None,
                                   ptr(st) if want_obj else None, C.byref(ns)))
    return obj, st, ns.value


@dataclass
class sdEpigraphInfo:
    """epigraph.jl:152-171: the cuts, incumbent cut and total weight of an epigraph at one
    moment (copies), for the incumbent test of the next step."""
    objective_weight: float
    cuts: list
    incumbent_cut: object
    total_scenario_weight: float
    lower_bound: float

    @classmethod
    def of(cls, epi: "sdEpigraph") -> "sdEpigraphInfo":
        return cls(epi.objective_weight, list(epi.cuts), epi.incumbent_cut, epi.total_scenario_weight,
                   epi.lower_bound)


def sd_iteration_solve(epis, scenario_values, x_candidate, x_incumbent, V: sdDualVertexSet):
    """algorithm.jl:45-55: for every epigraph i, add_scenario!(epi_i, w_i, 1.0), solve at
    x_candidate and at x_incumbent and push! both duals.  The duals are pushed in the
    reference's order (epi 1 cand, epi 1 inc, epi 2 cand, ...; for a block of several
    scenarios per epigraph: cand/inc per scenario in order).  scenario_values[i] is a
    (N_i x k) block of new scenarios for epigraph i.  Returns the vertex index of every
    pushed dual (the order above)."""
    pis = []
    for epi, vals in zip(epis, scenario_values):
        vals = np.atleast_2d(vals)
        first = epi.num_scenarios
        add_scenarios(epi, vals, np.ones(vals.shape[0]))
        _, _, pc, _ = solve_batch(epi, x_candidate, first, vals.shape[0])
        _, _, pinc, _ = solve_batch(epi, x_incumbent, first, vals.shape[0])
        inter = np.empty((2 * vals.shape[0], pc.shape[1]))
        inter[0::2] = pc
        inter[1::2] = pinc
        pis.append(inter)
    return V.push_batch(np.vstack(pis))


def sd_iteration_cuts(epis, x_candidate, x_incumbent, V: sdDualVertexSet, update_incumbent_cut=True,
                      tie_rel=DEFAULT_TIE_REL):
    """algorithm.jl:79-85: build_sasa_cut at x_candidate appended to epi.cuts and, if
    update_incumbent_cut, at x_incumbent as epi.incumbent_cut."""
    for epi in epis:
        epi.cuts.append(build_sasa_cut(epi, x_candidate, V, tie_rel))
        if update_incumbent_cut:
            epi.incumbent_cut = build_sasa_cut(epi, x_incumbent, V, tie_rel)


def sd_iteration_hot_path(epis, scenario_values, x_candidate, x_incumbent, V: sdDualVertexSet,
                          update_incumbent_cut=True, tie_rel=DEFAULT_TIE_REL):
    """The data-parallel part of sd_iteration! (algorithm.jl:45-55 and :79-85) in one call:
    sd_iteration_solve, the sdEpigraphInfo snapshot the reference takes between the two
    halves (algorithm.jl:76: after add_scenario!, before any new cut), sd_iteration_cuts.
    Returns the snapshot (epi_info_last) for check_improvement.  Cut removal by master
    multipliers (algorithm.jl:57-72) sits between the halves in the reference; callers with
    a master use the two halves directly (sqlp_amd.master.sd_iteration)."""
    sd_iteration_solve(epis, scenario_values, x_candidate, x_incumbent, V)
    info = [sdEpigraphInfo.of(e) for e in epis]
    sd_iteration_cuts(epis, x_candidate, x_incumbent, V, update_incumbent_cut, tie_rel)
    return info

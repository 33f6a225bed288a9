"""Master side of an SD iteration and the extensive form.

Reference -> here:
  sdCell(root_prob)                       cell.jl:44-71        -> sdCell(sp1)
  bind_epigraph!(cell, epi)               cell.jl:99-116       -> sdCell.bind_epigraph
  add_regularization!(cell, x0, rho)      cell.jl:130-134      -> sdCell.add_regularization
  sync_cuts!(cell)                        cell.jl:167-201      -> sdCell.sync_cuts (cut_pool.sdMasterCuts)
  optimize!(cell.master) / value.(x_ref)  algorithm.jl:100-112 -> sdCell.solve_master
  sd_iteration!(cell, scenario_list; ...) algorithm.jl:39-115  -> sd_iteration
  ConstantQuadScalarSchedule /            quad_scalar.jl:4-75  -> same names
    AdaptiveQuadScalarSchedule
  all_in_one(sp1, sp2, scenarios, probs)  crash.jl:18-72       -> all_in_one
  check_first_stage_feasible(sp1, x)      prob.jl:20-32        -> check_first_stage_feasible

The master is a small dense problem (n1 + E variables, m1 + #cuts rows; storm 126 x ~400)
that is not data-parallel, so it runs on the host: a primal-dual interior-point method
(Mehrotra predictor-corrector) for the convex QP

    min 1/2 z'Hz + g'z   s.t.   A z = b,   G z <= h

with dense LAPACK solves of the reduced KKT system.  The reference hands the same model to
CPLEX (instance drivers) or GLPK (the LP-only unit tests); like them it returns the primal
point and the row multipliers the cut removal of algorithm.jl:57-72 reads (|dual| < 0.001).
The scenario subproblems and cuts of each iteration (algorithm.jl:45-55, 79-85) run on the
GPU through twosd.sd_iteration_solve / sd_iteration_cuts.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

from . import cut_pool, twosd
from .smps import spStageProblem

OPTIMAL = "OPTIMAL"
INFEASIBLE_OR_UNBOUNDED = "INFEASIBLE_OR_UNBOUNDED"
ITERATION_LIMIT = "ITERATION_LIMIT"


# ------------------------------------------------------------------ dense convex QP (IPM)
@dataclass
class QPResult:
    status: str
    z: np.ndarray
    y: np.ndarray        # multipliers of A z = b  (Lagrangian + y'(Az - b))
    lam: np.ndarray      # multipliers of G z <= h, >= 0
    obj: float
    iterations: int


def qp_solve(H, g, A, b, G, h, tol=1e-10, max_iter=200) -> QPResult:
    """Mehrotra predictor-corrector interior point for min 1/2 z'Hz + g'z, Az = b, Gz <= h.
    H: (n, n) PSD or (n,) diagonal.  Rows of A and G are scaled to unit inf-norm inside;
    the returned multipliers are those of the original rows."""
    g = np.asarray(g, dtype=np.float64)
    n = g.shape[0]
    Hm = np.diag(np.asarray(H, dtype=np.float64)) if np.ndim(H) == 1 else np.asarray(H, dtype=np.float64)
    A = np.zeros((0, n)) if A is None else np.atleast_2d(np.asarray(A, dtype=np.float64)).reshape(-1, n)
    b = np.zeros(0) if b is None else np.asarray(b, dtype=np.float64).reshape(-1)
    G = np.zeros((0, n)) if G is None else np.atleast_2d(np.asarray(G, dtype=np.float64)).reshape(-1, n)
    h = np.zeros(0) if h is None else np.asarray(h, dtype=np.float64).reshape(-1)
    # row scaling (the multipliers scale back at the end)
    sa = np.maximum(np.abs(A).max(axis=1), 1e-300) if A.shape[0] else np.ones(0)
    sg = np.maximum(np.abs(G).max(axis=1), 1e-300) if G.shape[0] else np.ones(0)
    A, b = A / sa[:, None], b / sa
    G, h = G / sg[:, None], h / sg
    me, mi = A.shape[0], G.shape[0]
    scale = max(1.0, np.abs(g).max(initial=0.0), np.abs(b).max(initial=0.0), np.abs(h).max(initial=0.0))
    z = np.zeros(n)
    y = np.zeros(me)
    s = np.maximum(h - G @ z, 1.0) if mi else np.zeros(0)
    lam = np.ones(mi)
    reg = 1e-12 * (1.0 + np.abs(Hm).max(initial=0.0))

    def kkt_solve(M, rz, rp):
        K = np.zeros((n + me, n + me))
        K[:n, :n] = M + reg * np.eye(n)
        K[:n, n:] = A.T
        K[n:, :n] = A
        K[n:, n:] = -reg * np.eye(me)
        try:
            sol = np.linalg.solve(K, np.concatenate([rz, rp]))
        except np.linalg.LinAlgError:
            sol = np.linalg.lstsq(K, np.concatenate([rz, rp]), rcond=None)[0]
        return sol[:n], sol[n:]

    status = ITERATION_LIMIT
    it = 0
    for it in range(1, max_iter + 1):
        rd = Hm @ z + g + A.T @ y + G.T @ lam
        rp = A @ z - b
        ri = G @ z + s - h
        mu = float(s @ lam) / mi if mi else 0.0
        obj = 0.5 * z @ Hm @ z + g @ z
        if (np.abs(rd).max(initial=0.0) <= tol * scale and np.abs(rp).max(initial=0.0) <= tol * scale
                and np.abs(ri).max(initial=0.0) <= tol * scale and mu * mi <= tol * (1.0 + abs(obj))):
            status = OPTIMAL
            break
        if mi and (np.abs(z).max() > 1e14 or lam.max() > 1e14):
            status = INFEASIBLE_OR_UNBOUNDED
            break
        w = lam / s if mi else np.zeros(0)
        M = Hm + (G.T * w) @ G if mi else Hm

        def direction(rc):
            # rc: complementarity rhs (Lambda ds + S dlam = rc)
            rz = -rd - (G.T @ ((rc + lam * ri) / s) if mi else 0.0)
            dz, dy = kkt_solve(M, rz, -rp)
            dlam = (rc + lam * ri + lam * (G @ dz)) / s if mi else np.zeros(0)
            ds = -ri - G @ dz if mi else np.zeros(0)
            return dz, dy, dlam, ds

        def step_len(v, dv):
            neg = dv < 0
            return min(1.0, float(np.min(-v[neg] / dv[neg]))) if neg.any() else 1.0

        if not mi:
            dz, dy, _, _ = direction(np.zeros(0))
            z, y = z + dz, y + dy
            continue
        # predictor
        dz, dy, dlam, ds = direction(-s * lam)
        ap = step_len(s, ds)
        ad = step_len(lam, dlam)
        mu_aff = float((s + ap * ds) @ (lam + ad * dlam)) / mi
        sigma = (mu_aff / mu) ** 3 if mu > 0 else 0.0
        # corrector
        dz, dy, dlam, ds = direction(-s * lam + sigma * mu - ds * dlam)
        ap = 0.99 * step_len(s, ds)
        ad = 0.99 * step_len(lam, dlam)
        z = z + ap * dz
        s = s + ap * ds
        y = y + ad * dy
        lam = lam + ad * dlam
    obj = 0.5 * z @ Hm @ z + g @ z
    return QPResult(status, z, y / sa if me else y, lam / sg if mi else lam, float(obj), it)


# ------------------------------------------------------------------ stage-1 problem pieces
def _stage1_rows(sp1: spStageProblem):
    """(A1 dense, b1, sense1) of the root-stage rows (smps_prob.jl:65-100, stage 1)."""
    A1 = sp1.dense_W()
    return A1, np.asarray(sp1.r, dtype=np.float64), list(sp1.sense)


def _split_rows(A, b, sense):
    """Rows by sense -> (A_eq, b_eq, G, h) with G z <= h."""
    eq = [i for i, s in enumerate(sense) if s == "E"]
    le = [i for i, s in enumerate(sense) if s == "L"]
    ge = [i for i, s in enumerate(sense) if s == "G"]
    G = np.vstack([A[le], -A[ge]]) if (le or ge) else np.zeros((0, A.shape[1]))
    h = np.concatenate([b[le], -b[ge]]) if (le or ge) else np.zeros(0)
    return A[eq], b[eq], G, h


def _bound_rows(lb, ub, n_total, offset=0):
    """Finite variable bounds as G z <= h rows over n_total variables."""
    rows, rhs = [], []
    for j, (lo, hi) in enumerate(zip(lb, ub)):
        if np.isfinite(lo):
            r = np.zeros(n_total); r[offset + j] = -1.0
            rows.append(r); rhs.append(-lo)
        if np.isfinite(hi):
            r = np.zeros(n_total); r[offset + j] = 1.0
            rows.append(r); rhs.append(hi)
    return (np.array(rows).reshape(-1, n_total), np.array(rhs, dtype=np.float64))


def check_first_stage_feasible(sp1: spStageProblem, x, tol=1e-9) -> bool:
    """prob.jl:20-32: x satisfies the root-stage rows and bounds (a feasibility solve with x
    fixed is exactly this check)."""
    x = np.asarray(x, dtype=np.float64)
    A1, b1, sense = _stage1_rows(sp1)
    ax = A1 @ x
    sc = tol * (1.0 + np.abs(b1))
    for i, s in enumerate(sense):
        if (s == "G" and ax[i] < b1[i] - sc[i]) or (s == "L" and ax[i] > b1[i] + sc[i]) or \
                (s == "E" and abs(ax[i] - b1[i]) > sc[i]):
            return False
    return bool(np.all(x >= sp1.ylb - tol * (1 + np.abs(sp1.ylb))) and np.all(x <= sp1.yub + tol * (1 + np.abs(sp1.yub))))


def all_in_one(sp1: spStageProblem, sp2: spStageProblem, scenario_rhs, probs=None):
    """crash.jl:18-72: the deterministic equivalent over the given scenarios.
    scenario_rhs[s] is the stage-2 rhs r_s (m2; scenario values written into the template,
    instantiate!, smps_routines.jl:7-24); probs default 1/S.  Returns (obj, x, [y_s])."""
    S = len(scenario_rhs)
    probs = [1.0 / S] * S if probs is None else list(probs)
    A1, b1, sense1 = _stage1_rows(sp1)
    m1, n1 = A1.shape
    m2, n1b, n2 = sp2.shape
    assert n1b == n1, "sp2 last-stage variables must match sp1's current-stage variables (crash.jl:22)"
    W, T = sp2.dense_W(), sp2.dense_T()
    nz = n1 + S * n2
    g = np.concatenate([np.asarray(sp1.q, dtype=np.float64)] + [p * np.asarray(sp2.q) for p in probs])
    rows, rhs, sense = [np.hstack([A1, np.zeros((m1, S * n2))])], [b1], list(sense1)
    for s in range(S):
        blk = np.zeros((m2, nz))
        blk[:, :n1] = T
        blk[:, n1 + s * n2:n1 + (s + 1) * n2] = W
        rows.append(blk)
        rhs.append(np.asarray(scenario_rhs[s], dtype=np.float64))
        sense += list(sp2.sense)
    A = np.vstack(rows)
    bb = np.concatenate(rhs)
    Aeq, beq, G, h = _split_rows(A, bb, sense)
    lb = np.concatenate([sp1.ylb] + [sp2.ylb] * S)
    ub = np.concatenate([sp1.yub] + [sp2.yub] * S)
    Gb, hb = _bound_rows(lb, ub, nz)
    res = qp_solve(np.zeros(nz), g, Aeq, beq, np.vstack([G, Gb]), np.concatenate([h, hb]))
    if res.status != OPTIMAL:
        raise RuntimeError(f"all_in_one: extensive form not solved ({res.status})")
    x = res.z[:n1]
    ys = [res.z[n1 + s * n2:n1 + (s + 1) * n2] for s in range(S)]
    return res.obj, x, ys


# ------------------------------------------------------------------ quad-scalar schedules
def ConstantQuadScalarSchedule(reg: float):
    """quad_scalar.jl:4-7."""
    def g(cell):
        return reg
    return g


def AdaptiveQuadScalarSchedule(min_quad_scalar=1e-3, max_quad_scalar=1e4, R2=0.95, R3=2.0, tolerance=1e-3):
    """quad_scalar.jl:15-75 (state in cell.ext['quad_scalar'] / ['normDk_1'])."""
    def g(cell):
        if "quad_scalar" not in cell.ext:
            raise AssertionError("Quad_scalar not initialized. To use AdaptiveQuadScalarSchedule, "
                                 "set up cell.ext['quad_scalar'] first!")
        d = cell.x_incumbent - cell.x_candidate
        normDk = float(sum(v * v for v in d))
        if "normDk_1" not in cell.ext:
            if normDk > tolerance:
                cell.ext["normDk_1"] = normDk
            else:
                return cell.ext["quad_scalar"]
        normDk_1 = cell.ext["normDk_1"]
        if cell.improvement_info.is_improved:
            if normDk > tolerance and normDk >= R3 * normDk_1:
                cell.ext["quad_scalar"] *= R2 * R3 * normDk_1 / normDk
        else:
            cell.ext["quad_scalar"] /= R2
        cell.ext["quad_scalar"] = max(min(cell.ext["quad_scalar"], max_quad_scalar), min_quad_scalar)
        cell.ext["normDk_1"] = normDk
        return cell.ext["quad_scalar"]
    return g


# ------------------------------------------------------------------ the cell
class sdCell:
    """cell.jl:4-71: the master (root-stage rows, objective c'x + sum_e w_e eta_e, cuts,
    prox term), its epigraphs, the shared dual vertex set (on the GPU context) and the
    candidate / incumbent points."""

    def __init__(self, sp1: spStageProblem, ctx: twosd.SDContext):
        self.sp1 = sp1
        self.ctx = ctx
        self.A1, self.b1, self.sense1 = _stage1_rows(sp1)
        self.c1 = np.asarray(sp1.q, dtype=np.float64)
        self.n1 = self.A1.shape[1]
        self.epi: list = []
        self.dual_vertices = twosd.sdDualVertexSet(ctx)
        self.x_candidate = np.zeros(self.n1)
        self.x_incumbent = np.zeros(self.n1)
        self.improvement_info = None
        self.ext: dict = {}
        self.cuts = cut_pool.sdMasterCuts(0)
        self.reg_center = None
        self.rho = 0.0
        self.master_status = None      # termination status of the last master solve
        self.master_obj = None

    def objf_original(self, x) -> float:
        """evaluate_expr(cell.objf_original, x): the root-stage objective c'x."""
        return float(np.dot(self.c1, x))

    def bind_epigraph(self, epi: twosd.sdEpigraph):
        """cell.jl:99-116: new epigraph variable, weight objective_weight in the objective."""
        self.epi.append(epi)
        self.cuts.epicon_ref.append([])
        self.cuts.epicon_incumbent_ref.append(None)

    def add_regularization(self, x0, rho):
        """cell.jl:130-134: objective + sum_i rho/2 (x_i - x0_i)^2."""
        self.reg_center = np.array(x0, dtype=np.float64)
        self.rho = float(rho)

    def sync_cuts(self):
        """cell.jl:198-201."""
        self.cuts.sync_cuts(self.epi)

    def solve_master(self):
        """optimize!(cell.master) (algorithm.jl:104-112): returns x; stores the cut-row
        multipliers for the next iteration's cut removal."""
        E = len(self.epi)
        n1 = self.n1
        nz = n1 + E
        epi_rows, alpha, beta, _ = self.cuts.rows()
        for e in range(E):
            if not np.any(epi_rows == e):
                raise RuntimeError(f"epigraph {e} has no cut: the master is unbounded")
        H = np.zeros(nz)
        g = np.concatenate([self.c1, [e.objective_weight for e in self.epi]])
        if self.reg_center is not None and self.rho != 0.0:
            H[:n1] = self.rho
            g[:n1] -= self.rho * self.reg_center
        Aeq, beq, G, h = _split_rows(np.hstack([self.A1, np.zeros((self.A1.shape[0], E))]), self.b1, self.sense1)
        # cut rows: eta_e >= alpha + beta'x  <=>  beta'x - eta_e <= -alpha
        Gc = np.zeros((len(alpha), nz))
        if len(alpha):
            Gc[:, :n1] = beta
            Gc[np.arange(len(alpha)), n1 + epi_rows] = -1.0
        Gb, hb = _bound_rows(self.sp1.ylb, self.sp1.yub, nz)
        res = qp_solve(H, g, Aeq, beq, np.vstack([G, Gc, Gb]), np.concatenate([h, -alpha, hb]))
        self.master_status = res.status
        if res.status != OPTIMAL:
            raise RuntimeError(f"master not solved: {res.status}")
        lam = res.lam[G.shape[0]:G.shape[0] + len(alpha)]
        # multiplier of every master row, in master order, for remove_cuts_by_multiplier
        self._row_duals = lam
        const = 0.5 * self.rho * float(self.reg_center @ self.reg_center) if self.reg_center is not None else 0.0
        self.master_obj = res.obj + const
        return res.z[:n1].copy()

    def cut_duals(self):
        """Per epigraph, the multipliers of its non-incumbent cut rows (epicon_ref order)."""
        row_of = {id(r): i for i, r in enumerate(self.cuts._rows)}
        return [np.array([self._row_duals[row_of[id(r)]] for r in self.cuts.epicon_ref[e]])
                for e in range(len(self.epi))]


def sd_iteration(cell: sdCell, scenario_list, update_incumbent_cut=True, quad_scalar_schedule=None,
                 tie_rel=0.0):
    """sd_iteration! (algorithm.jl:39-115).  scenario_list[i] = element values (k) of the new
    scenario of epigraph i.  Steps 1-3 and 5-6 (the data-parallel hot segment) run on the GPU
    (twosd.sd_iteration_solve / sd_iteration_cuts); cut removal, incumbent selection,
    the prox schedule and the master solve run here."""
    if quad_scalar_schedule is None:
        quad_scalar_schedule = ConstantQuadScalarSchedule(0.1)
    assert len(scenario_list) == len(cell.epi)                        # algorithm.jl:42
    vals = [np.atleast_2d(np.asarray(v, dtype=np.float64)) for v in scenario_list]
    twosd.sd_iteration_solve(cell.epi, vals, cell.x_candidate, cell.x_incumbent, cell.dual_vertices)
    # remove cuts with small multipliers (algorithm.jl:57-72)
    if cell.master_status == OPTIMAL:
        cell.cuts.remove_cuts_by_multiplier(cell.epi, cell.cut_duals())
    epi_info_last = [twosd.sdEpigraphInfo.of(e) for e in cell.epi]    # algorithm.jl:76
    twosd.sd_iteration_cuts(cell.epi, cell.x_candidate, cell.x_incumbent, cell.dual_vertices,
                            update_incumbent_cut=update_incumbent_cut, tie_rel=tie_rel)
    cell.improvement_info = twosd.check_improvement(
        epi_info_last, cell.epi, cell.objf_original(cell.x_candidate), cell.objf_original(cell.x_incumbent),
        cell.x_candidate, cell.x_incumbent)
    rho = quad_scalar_schedule(cell)                                   # algorithm.jl:94
    if cell.improvement_info.is_improved:
        cell.x_incumbent = cell.x_candidate.copy()
    cell.add_regularization(cell.x_incumbent, rho)
    cell.sync_cuts()
    cell.x_candidate = cell.solve_master()

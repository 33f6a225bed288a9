"""1:1 ctypes restatement of julia/TwoSDHip.jl (test harness; Julia is not installed here).

Every function below is the Julia function of the same name in julia/TwoSDHip.jl: the same
C entry points in the same order, the same argument types (Cint / Int64 / Float64 / UInt8
pointers, declared as argtypes), the template and positions handed over 1-based
(index_base = 1, Julia's SparseMatrixCSC colptr / rowval as they are), scenario indices 0-based.

The Julia method wraps the reference's own objects, which do not exist in Python.  They are
stood in for by the build's host restatements:
  TwoSD.sdCell (JuMP master, epicon_ref, x's)          -> sqlp_amd.master.sdCell (host QP)
  TwoSD.sdEpigraph (cuts, weights, total weight)       -> RefEpigraph below
  TwoSD.add_scenario! / sdEpigraphInfo / check_improvement / sync_cuts! / add_regularization!
    / the cut removal by dual(con)                     -> RefEpigraph.add_scenario,
       twosd.sdEpigraphInfo.of, twosd.check_improvement, sdCell.sync_cuts /
       add_regularization / cut_duals
so `sd_iteration` below reads line for line like `TwoSD.sd_iteration!(hc::HipCell, ...)`.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field

import numpy as np

from sqlp_amd import _lib, master, twosd
from sqlp_amd.smps import spSmpsPosition

Cint, Int64, F64 = C.c_int, C.c_int64, C.c_double
P = C.c_void_p
PI32, PI64, PF64, PU8 = C.POINTER(Cint), C.POINTER(Int64), C.POINTER(F64), C.POINTER(C.c_uint8)

# ccall signatures of julia/TwoSDHip.jl (argument types as the Julia tuples declare them)
CCALLS = {
    "twosd_last_error": (C.c_char_p, []),
    "twosd_create": (Cint, [Cint, C.POINTER(P)]),
    "twosd_destroy": (Cint, [P]),
    "twosd_set_template": (Cint, [P, Cint, Cint, Cint, PI64, PI64, PF64, PI64, PI64, PF64, PF64, PF64, PU8,
                                  PF64, PF64, Cint]),
    "twosd_set_random_positions": (Cint, [P, Cint, PI32, PI32, Cint]),
    "twosd_compute_basis": (Cint, [P, PF64, PF64]),
    "twosd_solve_values": (Cint, [P, PF64, Cint, PF64, PF64, PF64, PF64, PI32]),
    "twosd_epigraph_create": (Cint, [P, PI32]),
    "twosd_add_scenarios": (Cint, [P, Cint, Cint, PF64, PF64]),
    "twosd_epigraph_info": (Cint, [P, Cint, PI32, PF64]),
    "twosd_solve_push": (Cint, [P, Cint, PF64, Cint, Cint, PF64, PI32, PI32]),
    "twosd_build_cut": (Cint, [P, Cint, PF64, F64, PF64, PF64, PF64, PF64, PI32]),
    "twosd_dvs_push": (Cint, [P, Cint, PF64, PI32, PI32]),
    "twosd_dvs_size": (Cint, [P, PI32]),
    "twosd_dvs_fingerprint": (Cint, [P, C.POINTER(C.c_uint64)]),
    "twosd_last_objective": (Cint, [P, PF64, PF64]),
}

_LIB = None


def LIB():
    global _LIB
    if _LIB is None:
        _lib.load()                                   # raises if the HIP library is not built
        lib = C.CDLL(_lib.LIB_PATH)                   # own handle: own argtypes
        for name, (res, args) in CCALLS.items():
            f = getattr(lib, name)
            f.restype, f.argtypes = res, args
        _LIB = lib
    return _LIB


def check(rc):
    if rc != 0:
        raise _lib.TwoSDError(rc, LIB().twosd_last_error().decode())


def _p(a, t):
    return a.ctypes.data_as(t)


def f64(a):
    return np.ascontiguousarray(a, dtype=np.float64)


# ------------------------------------------------------------------------------------------
# HipContext (TwoSDHip.jl: HipContext, element_values, compute_basis!, solve_problem)
class HipContext:
    def __init__(self, sp2, sto, device=0):
        ref = P()
        check(LIB().twosd_create(device, C.byref(ref)))
        self.h = ref
        m, n1, n2 = sp2.shape
        (Tcp, Trv, Tnz), (Wcp, Wrv, Wnz) = sp2.T, sp2.W
        # Julia SparseMatrixCSC arrays: Int64 colptr / rowval, 1-based
        self._keep = [np.ascontiguousarray(a + 1, dtype=np.int64) for a in (Tcp, Trv, Wcp, Wrv)]
        Tcp1, Trv1, Wcp1, Wrv1 = self._keep
        q, r = f64(sp2.q), f64(sp2.r)
        sense = np.frombuffer("".join(sp2.sense).encode(), dtype=np.uint8).copy()
        self._keep += [q, r, sense, f64(Tnz), f64(Wnz)]
        check(LIB().twosd_set_template(self.h, m, n1, n2, _p(Tcp1, PI64), _p(Trv1, PI64), _p(self._keep[7], PF64),
                                       _p(Wcp1, PI64), _p(Wrv1, PI64), _p(self._keep[8], PF64), _p(q, PF64),
                                       _p(r, PF64), _p(sense, PU8), None, None, 1))
        pos = list(sto.indep.keys())
        row_lookup = {nm: i + 1 for i, nm in enumerate(sp2.stage_constraints)}     # coef.row_lookup (1-based)
        col_lookup = {nm: j + 1 for j, nm in enumerate(sp2.last_stage_vars)}
        rows = np.array([row_lookup[p.row_name] for p in pos], dtype=np.int32)
        cols = np.array([-1 if p.col_name in ("RHS", "rhs") else col_lookup[p.col_name] for p in pos], dtype=np.int32)
        check(LIB().twosd_set_random_positions(self.h, len(pos), _p(rows, PI32), _p(cols, PI32), 1))
        self.nrow, self.n1, self.n2 = m, n1, n2
        self.positions = pos
        self.has_basis = False

    def close(self):
        if self.h:
            LIB().twosd_destroy(self.h)
            self.h = None

    __del__ = close


def element_values(ctx: HipContext, scenario) -> np.ndarray:
    d = {spSmpsPosition(*p): v for p, v in scenario}
    return np.array([d[p] for p in ctx.positions], dtype=np.float64)


def compute_basis(ctx: HipContext, x, scenario):
    v = element_values(ctx, scenario)
    check(LIB().twosd_compute_basis(ctx.h, _p(f64(x), PF64), _p(v, PF64)))
    ctx.has_basis = True


def solve_problem(ctx: HipContext, x, scenario):
    obj, st = F64(), Cint()
    y, pi = np.zeros(ctx.n2), np.zeros(ctx.nrow)
    v = element_values(ctx, scenario)
    check(LIB().twosd_solve_values(ctx.h, _p(f64(x), PF64), 1, _p(v, PF64), C.byref(obj), _p(pi, PF64),
                                   _p(y, PF64), C.byref(st)))
    return obj.value, y, pi


# ------------------------------------------------------------------------------------------
# HipEpigraph, HipDualVertexSet
class HipEpigraph:
    def __init__(self, ctx: HipContext):
        e = Cint()
        check(LIB().twosd_epigraph_create(ctx.h, C.byref(e)))
        self.ctx, self.index = ctx, e.value


def add_scenario(epi: HipEpigraph, scenario, weight=1.0):
    w = F64(weight)
    check(LIB().twosd_add_scenarios(epi.ctx.h, epi.index, 1, _p(element_values(epi.ctx, scenario), PF64), C.byref(w)))


def num_scenarios(epi: HipEpigraph) -> int:
    n = Cint()
    check(LIB().twosd_epigraph_info(epi.ctx.h, epi.index, C.byref(n), None))
    return n.value


def solve_push(epi: HipEpigraph, x, first, count) -> int:
    n = Cint()
    check(LIB().twosd_solve_push(epi.ctx.h, epi.index, _p(f64(x), PF64), first, count, None, None, C.byref(n)))
    return n.value


def last_objective(ctx: HipContext):
    a, b = F64(), F64()
    check(LIB().twosd_last_objective(ctx.h, C.byref(a), C.byref(b)))
    return a.value, b.value


def build_sasa_cut(epi: HipEpigraph, x, tie_rel=0.0) -> twosd.sdCut:
    a, wm = F64(), F64()
    beta = np.zeros(epi.ctx.n1)
    check(LIB().twosd_build_cut(epi.ctx.h, epi.index, _p(f64(x), PF64), tie_rel, C.byref(a), _p(beta, PF64),
                                C.byref(wm), None, None))
    return twosd.sdCut(a.value, beta, wm.value)


class HipDualVertexSet:
    def __init__(self, ctx: HipContext):
        self.ctx = ctx

    def push(self, pi):
        n = Cint()
        check(LIB().twosd_dvs_push(self.ctx.h, 1, _p(f64(pi), PF64), None, C.byref(n)))
        return self

    def __len__(self):
        n = Cint()
        check(LIB().twosd_dvs_size(self.ctx.h, C.byref(n)))
        return n.value

    def fingerprint(self):
        d = C.c_uint64()
        check(LIB().twosd_dvs_fingerprint(self.ctx.h, C.byref(d)))
        return d.value


# ------------------------------------------------------------------------------------------
# Stand-in for the reference's sdEpigraph (epigraph.jl:17-61): host record only
@dataclass
class RefEpigraph:
    objective_weight: float
    lower_bound: float
    scenario_list: list = field(default_factory=list)
    scenario_weight: list = field(default_factory=list)
    total_scenario_weight: float = 0.0
    cuts: list = field(default_factory=list)
    incumbent_cut: object = None

    def add_scenario(self, scenario, weight=1.0):
        """TwoSD.add_scenario! (epigraph.jl:81-96) without the host delta (unused here)."""
        self.scenario_list.append(scenario)
        self.scenario_weight.append(weight)
        self.total_scenario_weight += weight


# ------------------------------------------------------------------------------------------
# HipCell + sd_iteration! (TwoSDHip.jl: HipCell, TwoSD.sd_iteration!(hc::HipCell, ...))
class HipCell:
    def __init__(self, cell: master.sdCell, sp2, sto, device=0, tie_rel=0.0):
        if not cell.epi:
            raise RuntimeError("HipCell: bind the epigraphs first (bind_epigraph!)")
        self.cell = cell
        self.ctx = HipContext(sp2, sto, device=device)
        self.hepi = [HipEpigraph(self.ctx) for _ in cell.epi]
        for h, epi in zip(self.hepi, cell.epi):
            for w, wt in zip(epi.scenario_list, epi.scenario_weight):
                add_scenario(h, w, wt)
        self.dual_vertices = HipDualVertexSet(self.ctx)
        self.tie_rel = tie_rel

    def __getattr__(self, s):                  # Base.getproperty forwarding to the reference cell
        return getattr(self.__dict__["cell"], s)


def sd_iteration(hc: HipCell, scenario_list, update_incumbent_cut=True, quad_scalar_schedule=None):
    if quad_scalar_schedule is None:
        quad_scalar_schedule = master.ConstantQuadScalarSchedule(0.1)
    cell = hc.cell
    assert len(scenario_list) == len(cell.epi)                                       # :42
    if not hc.ctx.has_basis:
        compute_basis(hc.ctx, cell.x_candidate, scenario_list[0])

    for i in range(len(scenario_list)):                                              # :45-55
        cell.epi[i].add_scenario(scenario_list[i], 1.0)
        add_scenario(hc.hepi[i], scenario_list[i], 1.0)
        s = num_scenarios(hc.hepi[i]) - 1
        solve_push(hc.hepi[i], cell.x_candidate, s, 1)
        solve_push(hc.hepi[i], cell.x_incumbent, s, 1)

    if cell.master_status == master.OPTIMAL:                                         # :57-72
        duals = cell.cut_duals()
        for i in range(len(cell.cuts.epicon_ref)):
            delete_index = [j for j in range(len(cell.cuts.epicon_ref[i]))
                            if abs(duals[i][j]) < master.cut_pool.CUT_REMOVE_TOLERANCE]
            cell.epi[i].cuts[:] = [c for j, c in enumerate(cell.epi[i].cuts) if j not in set(delete_index)]

    epi_info_last = [twosd.sdEpigraphInfo.of(epi) for epi in cell.epi]              # :76

    for i, epi in enumerate(cell.epi):                                               # :79-85
        epi.cuts.append(build_sasa_cut(hc.hepi[i], cell.x_candidate, tie_rel=hc.tie_rel))
        if update_incumbent_cut:
            epi.incumbent_cut = build_sasa_cut(hc.hepi[i], cell.x_incumbent, tie_rel=hc.tie_rel)

    cell.improvement_info = twosd.check_improvement(                                 # :89-90
        epi_info_last, cell.epi, cell.objf_original(cell.x_candidate), cell.objf_original(cell.x_incumbent),
        cell.x_candidate, cell.x_incumbent)
    rho = quad_scalar_schedule(cell)                                                 # :94
    if cell.improvement_info.is_improved:
        cell.x_incumbent[:] = cell.x_candidate
    cell.add_regularization(cell.x_incumbent, rho)                                   # :101-102
    cell.sync_cuts()
    cell.x_candidate[:] = cell.solve_master()                                        # :104-112

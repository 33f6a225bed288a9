"""The Julia drop-in, exercised through its 1:1 ctypes mirror (tests/julia_mirror.py), against
an oracle replay of the whole sd_iteration! (algorithm.jl:39-115), SURVEY.md §8 rows b, a10, f3.

Per iteration the mirror runs TwoSDHip's `sd_iteration!(hc::HipCell, ...)` call sequence
(1-based template, device add / solve_push / build_cut, host master).  The replay repeats the
iteration on the oracle from the same x_candidate / x_incumbent and the same master
multipliers (so the test pins the bookkeeping, not the QP):
  * add_scenario!, solve at candidate and incumbent (C dual simplex, same start basis and pivot
    rules), push! (oracle/twosd_ref.py, dual_set.jl:84-94);
  * cut removal by multiplier (algorithm.jl:57-72) with the multipliers the mirror's master
    returned at the end of the previous iteration;
  * the sdEpigraphInfo snapshot (:76), build_sasa_cut at candidate and incumbent (:79-85);
  * check_improvement (:89-90), the incumbent update (:96-98), sync_cuts! with discounting
    (cell.jl:167-201, epigraph.jl:101-117).
Checked after every iteration: the vertex set in insertion order, every epigraph's cut list
(which cuts survived, alpha / beta to 1e-8 rel), the incumbent cut, the incumbent decision and
x_incumbent, and the master rows sync_cuts! wrote.

Ties: with the shim's default tie_rel = 0 (the reference's strict '>', subprob.jl:156) a
scenario whose two best vertex scores agree to ~1e-9 may pick either vertex, depending on the
summation order (GPU MFMA order vs the reference's dot order).  For such a cut the test checks
the tie-invariant value alpha + beta'x = sum p_w max_val_w, and the replay adopts the GPU cut.
With tie_rel = 1e-12 both sides apply the same near-tie rule and alpha / beta are compared for
every cut.
"""
import ctypes as C

import numpy as np
import pytest

from tests import instances as I

pytestmark = pytest.mark.gpu


def _scenario(positions, values):
    return [(p, float(v)) for p, v in zip(positions, values)]


def _device_vertices(hc):
    from sqlp_amd import _lib
    lib = _lib.load()
    n = len(hc.dual_vertices)
    out = np.zeros((n, hc.ctx.nrow))
    _lib.check(lib.twosd_dvs_get(hc.ctx.h, 0, n, out.ctypes.data_as(C.c_void_p)))
    return out


def _device_basis(hc):
    from sqlp_amd import _lib
    head = np.zeros(hc.ctx.nrow, dtype=np.int32)
    _lib.check(_lib.load().twosd_get_basis(hc.ctx.h, head.ctypes.data_as(C.c_void_p)))
    return head


def _near_tie(coef, deltas, x, Vm):
    base = coef.rhs - coef.transfer @ x
    for dr, dT in deltas:
        s = Vm @ (base + dr - dT @ x)
        if len(s) > 1:
            t = np.sort(s)[-2:]
            if t[1] - t[0] <= 1e-9 * (1 + abs(t[1])):
                return True
    return False


def _cell(name, E, seed=1):
    from sqlp_amd import master, smps
    from tests import julia_mirror as jm
    inst = I.load(name)
    sp1 = smps.get_smps_stage_template(inst["cor"], inst["tim"], 1)
    sp2 = inst["sp2"]
    if name == "lands":
        # starting point as the reference driver: extensive form over 10 sampled scenarios
        # (sd_single_cut_test.jl:40-46)
        row = sp2.stage_constraints.index("S2C5")
        rhs = []
        for v in I.sample("lands", 10, seed)[:, 0]:
            r = sp2.r.copy(); r[row] = v; rhs.append(r)
        _, x0, _ = master.all_in_one(sp1, sp2, rhs)
    else:
        x0 = I.x_ev(name)
    cell = master.sdCell(sp1, None)
    for _ in range(E):
        cell.bind_epigraph(jm.RefEpigraph(1.0 / E, 0.0))
    cell.x_candidate = np.array(x0, dtype=np.float64)
    cell.x_incumbent = np.array(x0, dtype=np.float64)
    return jm.HipCell(cell, sp2, inst["sto"]), sp1


@pytest.mark.parametrize("name,E,iters,tie_rel", [("lands", 1, 12, 0.0), ("lands", 1, 12, 1e-12),
                                                  ("transship", 2, 6, 0.0)])
def test_julia_mirror_sd_iteration_replay(name, E, iters, tie_rel):
    from oracle import cpu, twosd_ref
    from sqlp_amd import master
    from tests import julia_mirror as jm
    hc, sp1 = _cell(name, E)
    hc.tie_rel = tie_rel
    cell = hc.cell
    inst = I.load(name)
    sp = inst["osp2"]
    coef = twosd_ref.Coefficients(sp)
    positions = hc.ctx.positions
    rows = np.array([coef.row_lookup[p.row_name] for p in positions])
    oV = twosd_ref.DualVertexSet()
    o_deltas = [[] for _ in range(E)]
    o_cuts = [[] for _ in range(E)]
    o_inc = [None] * E
    lp = None
    c1 = np.asarray(sp1.q, dtype=np.float64)
    removed = 0
    ties = 0
    for it in range(iters):
        xc, xi = cell.x_candidate.copy(), cell.x_incumbent.copy()
        duals = cell.cut_duals() if cell.master_status == master.OPTIMAL else None
        vals = [I.sample(name, 1, 100 * it + e)[0] for e in range(E)]
        jm.sd_iteration(hc, [_scenario(positions, v) for v in vals])
        # ---- replay on the oracle --------------------------------------------------------
        if lp is None:
            lp = cpu.CpuLP(sp.W, sp.q, sp.senses)
            lp.set_basis(_device_basis(hc))
        for e in range(E):                                           # algorithm.jl:45-55
            o_deltas[e].append(twosd_ref.delta_coefficients(coef, list(zip(positions, vals[e]))))
            for x in (xc, xi):
                o_obj, o_pi, _, o_st, _ = lp.solve_batch(rows, sp.r - sp.T @ x, vals[e][None, :] - sp.r[rows],
                                                         nthreads=1)
                assert (o_st == 0).all()
                oV.push(o_pi[0])
        if duals is not None:                                        # algorithm.jl:57-72
            for e in range(E):
                before = len(o_cuts[e])
                o_cuts[e] = twosd_ref.remove_cuts_by_multiplier(o_cuts[e], duals[e])
                removed += before - len(o_cuts[e])
        tw = [float(len(o_deltas[e])) for e in range(E)]
        f_last = [(1.0 / E, list(o_cuts[e]), o_inc[e], tw[e], 0.0) for e in range(E)]   # :76
        Vm = oV.matrix()
        for e in range(E):                                           # :79-85
            w = np.ones(len(o_deltas[e]))
            for x, got in ((xc, cell.epi[e].cuts[-1]), (xi, cell.epi[e].incumbent_cut)):
                a, b, wm, mv, _ = twosd_ref.build_sasa_cut(coef, o_deltas[e], w, x, oV, tie_rel=tie_rel)
                assert got.weight_mark == wm
                val = float(np.sum(w / w.sum() * mv))
                assert got.alpha + got.beta @ x == pytest.approx(val, rel=1e-9, abs=1e-9)
                if _near_tie(coef, o_deltas[e], x, Vm):
                    ties += 1                                        # decided in the restatement's arithmetic
                assert got.alpha == pytest.approx(a, rel=1e-8, abs=1e-8)
                np.testing.assert_allclose(got.beta, b, rtol=1e-8, atol=1e-8 * (1 + np.abs(b).max()))
                if x is xc:
                    o_cuts[e].append((a, b, wm))
                else:
                    o_inc[e] = (a, b, wm)
        f_cur = [(1.0 / E, list(o_cuts[e]), o_inc[e], tw[e], 0.0) for e in range(E)]
        ce, ie, rq, imp = twosd_ref.check_improvement(f_last, f_cur, xc, xi, float(c1 @ xc), float(c1 @ xi))
        info = cell.improvement_info                                 # :89-90
        assert info.candidate_estimation == pytest.approx(ce, rel=1e-8, abs=1e-8)
        assert info.incumbent_estimation == pytest.approx(ie, rel=1e-8, abs=1e-8)
        assert info.is_improved == imp
        np.testing.assert_array_equal(cell.x_incumbent, xc if imp else xi)      # :96-98
        # ---- compare the state after the iteration ----------------------------------------
        assert len(hc.dual_vertices) == len(oV), (it, len(hc.dual_vertices), len(oV))
        np.testing.assert_allclose(_device_vertices(hc), Vm, rtol=1e-9, atol=1e-9)
        for e in range(E):
            assert len(cell.epi[e].cuts) == len(o_cuts[e])
            for got, (a, b, wm) in zip(cell.epi[e].cuts, o_cuts[e]):
                assert got.weight_mark == wm
                assert got.alpha == pytest.approx(a, rel=1e-8, abs=1e-8)
                np.testing.assert_allclose(got.beta, b, rtol=1e-8, atol=1e-8 * (1 + np.abs(b).max()))
            assert cell.epi[e].total_scenario_weight == tw[e]
        o_rows = twosd_ref.sync_cuts([(o_cuts[e], o_inc[e], tw[e], 0.0) for e in range(E)])   # cell.jl:167-201
        epi_rows, alpha, beta, inc = cell.cuts.rows()
        assert len(o_rows) == len(alpha)
        for r, (e, na, nb, isinc) in enumerate(o_rows):
            assert epi_rows[r] == e and bool(inc[r]) == isinc
            assert alpha[r] == pytest.approx(na, rel=1e-8, abs=1e-8)
            np.testing.assert_allclose(beta[r], nb, rtol=1e-8, atol=1e-8 * (1 + np.abs(nb).max()))
        assert master.check_first_stage_feasible(sp1, cell.x_candidate, tol=1e-7)
    assert removed > 0, "no cut was removed by multiplier: the replay did not exercise algorithm.jl:57-72"
    print(f"{name}: {iters} iterations, |V| = {len(oV)}, cuts removed {removed}, near-tie cuts {ties}")


def test_julia_mirror_passes_one_based_template():
    """The mirror hands the template and positions over 1-based, Int64 (index_base = 1) exactly
    as the Julia shim passes SparseMatrixCSC arrays; the device then solves like the 0-based
    product path (sqlp_amd.twosd)."""
    from sqlp_amd import smps, twosd
    from tests import julia_mirror as jm
    inst = I.load("storm")
    x = I.x_ev("storm")
    hctx = jm.HipContext(inst["sp2"], inst["sto"])
    mean = smps.mean_values(inst["sto"])
    jm.compute_basis(hctx, x, _scenario(hctx.positions, mean))
    ctx = twosd.SDContext(inst["sp2"], inst["sto"])
    ctx.compute_basis(x, mean)
    vals = I.sample("storm", 4, 3)
    for v in vals:
        o1, y1, pi1 = jm.solve_problem(hctx, x, _scenario(hctx.positions, v))
        o0, y0, pi0 = twosd.solve_problem(ctx, x, _scenario(ctx.positions, v))
        assert o1 == o0
        np.testing.assert_array_equal(pi1, pi0)

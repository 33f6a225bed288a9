"""CPU oracle: the pool warm start (oracle_lp_solve_batch_pool, the CPU counterpart of the
GPU basis pool used by bench.py's pooled cpu_baseline) reaches the same optimal objectives
as the single-basis warm start, with a per-scenario start chosen by least primal
infeasibility."""
import numpy as np
import pytest

from tests import instances as I


@pytest.mark.parametrize("name", ["transship", "ssn"])
def test_pool_warm_start_same_objectives(name):
    from oracle import cpu
    inst = I.load(name)
    sp = inst["osp2"]
    x = I.x_ev(name)
    base = sp.r - sp.T @ x
    from sqlp_amd import smps
    pos, rows, cols = smps.scenario_positions(inst["sp2"], inst["sto"])
    lp = cpu.CpuLP(sp.W, sp.q, sp.senses)
    train = I.sample(name, 6, seed=3)
    heads = []
    for v in train:
        b = base.copy()
        b[rows] += v - sp.r[rows]
        st, _, head, _ = lp.solve_from_slack(b)
        assert st == 0
        heads.append(head)
    lp.set_basis(heads[0])
    lp.set_pool(np.array(heads))
    vals = I.sample(name, 400, seed=9)
    DR = vals - sp.r[rows]
    o1, _, _, s1, it1 = lp.solve_batch(rows, base, DR, nthreads=4)
    o2, pi2, s2, it2, picks = lp.solve_batch_pool(rows, base, DR, nthreads=4)
    assert (s1 == 0).all() and (s2 == 0).all()
    np.testing.assert_allclose(o2, o1, rtol=1e-9, atol=1e-9)
    b_all = np.tile(base, (len(vals), 1))
    b_all[:, rows] += DR
    np.testing.assert_allclose(np.einsum("ij,ij->i", pi2, b_all), o2, rtol=1e-9, atol=1e-9)   # strong duality
    assert it2.mean() <= 1.5 * it1.mean()             # a heuristic start: pivots comparable, never required fewer
    assert picks.min() >= 0 and picks.max() < len(heads)

"""Host cut-pool bookkeeping against the reference's own KATs
(test/sd_test.jl:152-187) and the oracle's discount restatement (oracle/twosd_ref.py).
No device calls."""
import numpy as np
import pytest

from oracle import twosd_ref


class _Epi:   # the fields of sdEpigraph that the cut pool reads (epigraph.jl:17-61)
    def __init__(self, cuts, inc, tw, lb):
        self.cuts, self.incumbent_cut = list(cuts), inc
        self.total_scenario_weight, self.lower_bound = tw, lb


def _cuts():
    from sqlp_amd.twosd import sdCut
    c1 = sdCut(1.0, np.array([2.0, 3, 4, 5]), 1.0)
    c2 = sdCut(6.0, np.array([7.0, 8, 9, 10]), 2.0)
    inc = sdCut(11.0, np.array([12.0, 13, 14, 15]), 1.0)
    return c1, c2, inc


def test_add_cut_to_master_kat():
    """sd_test.jl:152-157: discount 1, lb 0 -> eta - [2,3,4,5]'x >= 1."""
    from sqlp_amd.cut_pool import add_cut_to_master, sdMasterCuts
    from sqlp_amd.twosd import sdCut
    m = sdMasterCuts(2)
    row = add_cut_to_master(m, sdCut(1.0, np.array([2.0, 3, 4, 5]), 0.1), 0, 1.0, 0.0)
    assert row.alpha == 1.0 and np.array_equal(row.beta, [2.0, 3, 4, 5]) and row.sense == "MIN_SENSE"
    assert m.is_valid(row)


def test_remove_cuts_kat():
    """sd_test.jl:159-164: a registered row is deleted and epicon_ref emptied."""
    from sqlp_amd.cut_pool import add_cut_to_master, sdMasterCuts
    c1, _, _ = _cuts()
    m = sdMasterCuts(2)
    con = add_cut_to_master(m, c1, 0, 1.0, 0.0)
    m.epicon_ref[0].append(con)
    m.remove_cuts(0)
    assert not m.is_valid(con) and m.epicon_ref[0] == []


def test_sync_cuts_kat():
    """sd_test.jl:166-187: two cuts + incumbent on epi 1, one cut on epi 2 (lb 100, total
    weight 2 -> discount 0.5, rhs 100*0.5 + 1*0.5 = 50.5); re-sync adds nothing twice."""
    from sqlp_amd.cut_pool import sdMasterCuts
    c1, c2, inc = _cuts()
    e1 = _Epi([c1, c2], inc, 2.0, 0.0)
    e2 = _Epi([c1], None, 2.0, 100.0)
    m = sdMasterCuts(2)
    m.sync_cuts(e1, 0)
    assert len(m.epicon_ref[0]) == 2 and m.epicon_incumbent_ref[0] is not None
    m.sync_cuts([e1, e2])
    assert len(m.epicon_ref[0]) == 2
    assert m.epicon_ref[1][0].alpha == 50.5
    epi, alpha, beta, incf = m.rows()
    assert list(epi) == [0, 0, 0, 1] and list(incf) == [False, False, True, False]
    # discounts weight_mark / total: c1 0.5, c2 1.0, incumbent 1.0 (cell.jl:174-189)
    assert np.array_equal(alpha, [0.5 * 1.0, 6.0, 11.0, 50.5])
    assert np.array_equal(beta[0], 0.5 * c1.beta) and np.array_equal(beta[2], inc.beta)


def test_sync_rows_match_oracle_and_evaluate():
    """Every synced row equals the oracle's add_cut_discount; the max over an epigraph's rows
    and its lower bound equals evaluate_epigraph (MIN sense) at random x."""
    from sqlp_amd import twosd
    from sqlp_amd.cut_pool import sdMasterCuts
    rng = np.random.default_rng(11)
    for _ in range(30):
        epis = []
        for _e in range(int(rng.integers(1, 4))):
            cuts = [twosd.sdCut(float(rng.normal()), rng.normal(size=5), float(rng.uniform(0.5, 3)))
                    for _ in range(int(rng.integers(0, 6)))]
            inc = twosd.sdCut(float(rng.normal()), rng.normal(size=5), 1.0) if rng.random() < 0.5 else None
            epis.append(_Epi(cuts, inc, float(rng.uniform(3, 5)), float(rng.normal())))
        m = sdMasterCuts(len(epis))
        m.sync_cuts(epis)
        for e, epi in enumerate(epis):
            for cut, row in zip(epi.cuts, m.epicon_ref[e]):
                a, b = twosd_ref.add_cut_discount(cut.alpha, cut.beta, cut.weight_mark / epi.total_scenario_weight,
                                                  epi.lower_bound)
                assert row.alpha == a and np.array_equal(row.beta, b)
            x = rng.normal(size=5)
            rows = m.epicon_ref[e] + ([m.epicon_incumbent_ref[e]] if epi.incumbent_cut is not None else [])
            best = epi.lower_bound
            for r in rows:
                best = max(best, r.alpha + float(np.dot(r.beta, x)))
            ref = twosd_ref.evaluate_epigraph([(c.alpha, c.beta, c.weight_mark) for c in epi.cuts],
                                              None if epi.incumbent_cut is None else
                                              (epi.incumbent_cut.alpha, epi.incumbent_cut.beta, 1.0),
                                              x, epi.total_scenario_weight, epi.lower_bound)
            assert best == pytest.approx(ref, rel=1e-14, abs=1e-14)


def test_remove_cuts_by_multiplier():
    """algorithm.jl:57-72: cuts whose master row has |dual| < 0.001 are deleted (by row
    index), the incumbent cut and cuts added after the last sync stay."""
    from sqlp_amd.cut_pool import sdMasterCuts
    from sqlp_amd.twosd import sdCut
    c1, c2, inc = _cuts()
    c3 = sdCut(3.0, np.array([1.0, 1, 1, 1]), 2.0)
    e1 = _Epi([c1, c2, c3], inc, 2.0, 0.0)
    e2 = _Epi([c1], None, 2.0, 100.0)
    m = sdMasterCuts(2)
    m.sync_cuts([e1, e2])
    late = sdCut(9.0, np.zeros(4), 2.0)
    e2.cuts.append(late)                                   # not yet synced
    m.remove_cuts_by_multiplier([e1, e2], [[0.0, 0.5, -0.0009], [-0.001]])
    assert e1.cuts == [c2] and e1.incumbent_cut is inc
    assert e2.cuts == [c1, late]                           # |-0.001| is not < 0.001
    with pytest.raises(ValueError):
        m.remove_cuts_by_multiplier([e1, e2], [[0.0], [0.0]])


def test_master_sense_max():
    """MAX-sense master: rows read eta <= alpha' + beta'x; unknown senses raise."""
    from sqlp_amd.cut_pool import MAX_SENSE, add_cut_to_master, sdMasterCuts
    c1, _, _ = _cuts()
    row = add_cut_to_master(sdMasterCuts(1, MAX_SENSE), c1, 0, 0.25, 8.0)
    assert row.sense == MAX_SENSE and row.alpha == 0.25 * 1.0 + 0.75 * 8.0
    with pytest.raises(ValueError):
        add_cut_to_master(sdMasterCuts(1, "FEASIBILITY"), c1, 0, 1.0, 0.0)


def test_sync_and_removal_match_oracle_restatement():
    """The product bookkeeping (sqlp_amd.cut_pool) vs the oracle's restatement of
    algorithm.jl:57-72 and cell.jl:167-201 on random multi-epigraph cut lists: the same cuts
    survive removal, and sync_cuts! writes the same master rows in the same order."""
    from sqlp_amd.cut_pool import sdMasterCuts
    from sqlp_amd.twosd import sdCut
    rng = np.random.default_rng(4)
    E, n1 = 3, 5
    epis, o_epis = [], []
    for e in range(E):
        tw = float(rng.integers(5, 20))
        cuts = [sdCut(float(rng.normal()), rng.normal(size=n1), float(rng.integers(1, int(tw) + 1)))
                for _ in range(int(rng.integers(2, 7)))]
        inc = sdCut(float(rng.normal()), rng.normal(size=n1), tw) if e != 1 else None
        lb = float(rng.normal())
        epis.append(_Epi(cuts, inc, tw, lb))
        o_epis.append(([(c.alpha, c.beta, c.weight_mark) for c in cuts], None if inc is None else
                       (inc.alpha, inc.beta, inc.weight_mark), tw, lb))
    m = sdMasterCuts(E)
    m.sync_cuts(epis)
    _check_rows(m, twosd_ref.sync_cuts(o_epis))
    # multipliers: about half below CUT_REMOVE_TOLERANCE (incl. negatives, exactly the tolerance)
    duals = [np.where(rng.random(len(m.epicon_ref[e])) < 0.5, rng.uniform(-9e-4, 9e-4, len(m.epicon_ref[e])),
                      rng.uniform(1e-3, 1.0, len(m.epicon_ref[e]))) for e in range(E)]
    duals[0][0] = 1e-3                                   # |dual| == tol is kept (strict '<')
    m.remove_cuts_by_multiplier(epis, duals)
    o_epis = [(twosd_ref.remove_cuts_by_multiplier(c, d), inc, tw, lb) for (c, inc, tw, lb), d in zip(o_epis, duals)]
    for epi, (c, _, _, _) in zip(epis, o_epis):
        assert [cut.alpha for cut in epi.cuts] == [a for a, _, _ in c]
    m.sync_cuts(epis)
    _check_rows(m, twosd_ref.sync_cuts(o_epis))


def _check_rows(m, o_rows):
    epi, alpha, beta, inc = m.rows()
    assert len(o_rows) == len(alpha)
    for r, (e, a, b, isinc) in enumerate(o_rows):
        assert epi[r] == e and bool(inc[r]) == isinc
        assert alpha[r] == a
        np.testing.assert_array_equal(beta[r], b)

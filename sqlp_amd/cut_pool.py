"""Host-side cut-pool bookkeeping around the hot path.

The reference keeps every epigraph's cuts in `epi.cuts` / `epi.incumbent_cut` and mirrors
them into the JuMP master as constraints `eta_e >= alpha' + beta'x`:

  add_cut_to_master!(master, cut, eta, x, discount, lb)   epigraph.jl:101-117
  remove_cuts!(cell, e) / remove_cuts!(cell)              cell.jl:139-161
  sync_cuts!(cell, epi, e) / sync_cuts!(cell)             cell.jl:167-201
  cut removal by master multiplier (|dual| < 0.001)       algorithm.jl:57-72

There is no JuMP here, so the master's epigraph rows are held in `sdMasterCuts` as plain
arrays (one row per constraint: epigraph index, alpha', beta', incumbent flag), in exactly
the order sync_cuts! adds them.  A master solver (outside this path: SURVEY.md §8 f4) reads
`rows()`; its row multipliers come back through `remove_cuts_by_multiplier`.  This is tiny,
sequential host work (a few hundred cuts of n1 doubles), so it stays in Python.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

from .twosd import MIN_SENSE, sdCut

# algorithm.jl:23
CUT_REMOVE_TOLERANCE = 0.001
MAX_SENSE = "MAX_SENSE"


@dataclass
class sdCutRow:
    """One epigraph constraint of the master: eta_e >= alpha + beta'x (MIN) or <= (MAX).
    As a JuMP row it reads eta_e - beta'x >= alpha, so `alpha` is its normalized rhs."""
    epi: int
    alpha: float
    beta: np.ndarray
    sense: str
    incumbent: bool = False


def add_cut_to_master(master: "sdMasterCuts", cut: sdCut, epi_num: int, discount: float,
                      lower_bound: float) -> sdCutRow:
    """add_cut_to_master! (epigraph.jl:101-117): alpha' = d*alpha + (1-d)*lb, beta' = d*beta;
    the row's direction follows the master's sense (>= for MIN, <= for MAX)."""
    if master.sense not in (MIN_SENSE, MAX_SENSE):
        raise ValueError("Unknown master sense. Master should either be MIN or MAX problem.")
    new_alpha = discount * cut.alpha + (1 - discount) * lower_bound
    new_beta = discount * np.asarray(cut.beta, dtype=np.float64)
    row = sdCutRow(int(epi_num), float(new_alpha), new_beta, master.sense)
    master._rows.append(row)
    return row


class sdMasterCuts:
    """The epigraph rows of a cell's master (the reference's cell.epicon_ref /
    cell.epicon_incumbent_ref, cell.jl:25-40), one list of cut rows per epigraph."""

    def __init__(self, num_epigraphs: int, sense: str = MIN_SENSE):
        self.sense = sense
        self._rows: list = []
        self.epicon_ref = [[] for _ in range(num_epigraphs)]
        self.epicon_incumbent_ref = [None] * num_epigraphs

    def is_valid(self, row: sdCutRow) -> bool:
        return any(r is row for r in self._rows)

    def delete(self, row: sdCutRow):
        for i, r in enumerate(self._rows):
            if r is row:
                del self._rows[i]
                return
        raise KeyError("constraint is not in the master")

    def remove_cuts(self, epi_num=None):
        """remove_cuts!(cell, e) (cell.jl:139-150); all epigraphs when epi_num is None
        (cell.jl:155-161)."""
        nums = range(len(self.epicon_ref)) if epi_num is None else [epi_num]
        for e in nums:
            for con in self.epicon_ref[e]:
                self.delete(con)
            self.epicon_ref[e].clear()
            if self.epicon_incumbent_ref[e] is not None:
                self.delete(self.epicon_incumbent_ref[e])
                self.epicon_incumbent_ref[e] = None

    def sync_cuts(self, epis, epi_num=None):
        """sync_cuts!(cell, epi, e) (cell.jl:167-192): drop epigraph e's rows, re-add every
        cut discounted by weight_mark / total_scenario_weight, then the incumbent cut with
        discount 1.  epi_num None = every epigraph in order (cell.jl:198-201); otherwise
        `epis` is the single epigraph for row set epi_num."""
        if epi_num is None:
            for e, epi in enumerate(epis):
                self.sync_cuts(epi, e)
            return
        epi = epis
        self.remove_cuts(epi_num)
        tw = epi.total_scenario_weight
        for cut in epi.cuts:
            con = add_cut_to_master(self, cut, epi_num, cut.weight_mark / tw, epi.lower_bound)
            self.epicon_ref[epi_num].append(con)
        if epi.incumbent_cut is not None:
            con = add_cut_to_master(self, epi.incumbent_cut, epi_num, 1.0, epi.lower_bound)
            con.incumbent = True
            self.epicon_incumbent_ref[epi_num] = con

    def rows(self):
        """(epi int32[R], alpha f64[R], beta f64[R, n1], incumbent bool[R]) in master order."""
        R = len(self._rows)
        n1 = len(self._rows[0].beta) if R else 0
        epi = np.array([r.epi for r in self._rows], dtype=np.int32)
        alpha = np.array([r.alpha for r in self._rows], dtype=np.float64)
        beta = np.zeros((R, n1)) if R else np.zeros((0, 0))
        for i, r in enumerate(self._rows):
            beta[i] = r.beta
        inc = np.array([r.incumbent for r in self._rows], dtype=bool)
        return epi, alpha, beta, inc

    def remove_cuts_by_multiplier(self, epis, duals, tol: float = CUT_REMOVE_TOLERANCE):
        """algorithm.jl:57-72: with the master solved, delete from epi.cuts every cut whose
        master row has |multiplier| < tol.  duals[e][j] is the multiplier of
        epicon_ref[e][j] (the j-th non-incumbent row of epigraph e); the incumbent cut is
        never deleted.  The master rows themselves are rebuilt by the next sync_cuts."""
        for e, epi in enumerate(epis):
            d = np.asarray(duals[e], dtype=np.float64)
            if d.shape[0] != len(self.epicon_ref[e]):
                raise ValueError(f"epigraph {e}: {d.shape[0]} multipliers for {len(self.epicon_ref[e])} cut rows")
            # deleteat! by row index j: cuts past the synced rows are untouched
            drop = {j for j, m in enumerate(d) if abs(m) < tol}
            epi.cuts[:] = [c for j, c in enumerate(epi.cuts) if j not in drop]

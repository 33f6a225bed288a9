"""SMPS reader + stage split (host plumbing that feeds the hot path).

Mirrors the reference's reader (names and semantics):
  read_cor                 src/smps/smps_cor.jl:160-194 (tokenizer :26-58, bounds :124-155)
  read_tim                 src/smps/smps_tim.jl:30-64
  read_sto                 src/smps/smps_sto.jl:41-110
  get_smps_stage_template  src/smps/smps_prob.jl:14-102
  rand(sto)                src/smps/smps_sto.jl:117-149 (DISCRETE / NORMAL(mean, variance) /
                           UNIFORM), here vectorised with numpy's PCG64 -- Julia's RNG
                           streams cannot be reproduced, so samples are not bitwise Julia's.
The product keeps everything sparse (CSC arrays ready for twosd_set_template).
"""
from __future__ import annotations

import os
from dataclasses import dataclass, field
from typing import NamedTuple

import numpy as np


class spSmpsPosition(NamedTuple):
    """(col_name, row_name) of a random element; col 'RHS'/'rhs' marks an RHS entry."""
    col_name: str
    row_name: str


@dataclass
class spCorType:
    problem_name: str
    directions: list
    row_names: list
    col_names: list
    entries: dict            # (row, col) -> value, last assignment wins
    rhs: np.ndarray
    lower_bound: np.ndarray
    upper_bound: np.ndarray
    col_mapping: dict
    row_mapping: dict


@dataclass
class spSmpsImplicitPeriod:
    period_name: str
    position: spSmpsPosition


@dataclass
class spTimType:
    problem_name: str
    periods: list


@dataclass
class spStoType:
    problem_name: str
    indep: dict = field(default_factory=dict)   # position -> (kind, a, b); insertion ordered


def _lines(path):
    with open(path, "r", encoding="latin-1") as f:
        return f.read().splitlines()


def read_cor(path) -> spCorType:
    sections = ("NAME", "ROWS", "COLUMNS", "RHS", "BOUNDS", "ENDATA")
    tok = {s: [] for s in sections}
    section = ""
    for line in _lines(path):
        if not line or line[0] == '*':
            continue
        t = line.split()
        if line[0] != ' ':
            section = t[0]
            if section not in sections:
                raise AssertionError(f"unsupported COR section {section!r}")
            if section == "NAME":
                tok["NAME"].append(t[1])          # BoundsError in the reference if missing
        else:
            tok[section].append(t)
    directions = [t[0][0] for t in tok["ROWS"]]
    row_names = [t[1] for t in tok["ROWS"]]
    col_names = list(dict.fromkeys(t[0] for t in tok["COLUMNS"]))
    rowm = {r: i for i, r in enumerate(row_names)}
    colm = {c: j for j, c in enumerate(col_names)}
    entries = {}
    for t in tok["COLUMNS"]:
        j = colm[t[0]]
        for a in range(1, len(t) - 1, 2):
            v = float(t[a + 1])
            key = (rowm[t[a]], j)
            if v != 0.0:
                entries[key] = v
            else:
                entries.pop(key, None)
    rhs = np.zeros(len(row_names))
    for t in tok["RHS"]:
        for a in range(1, len(t) - 1, 2):
            rhs[rowm[t[a]]] = float(t[a + 1])
    lb = np.zeros(len(col_names))
    ub = np.full(len(col_names), np.inf)
    for t in tok["BOUNDS"]:
        bt = t[0]
        if bt not in ("LO", "UP", "FX", "FR", "MI", "PL"):
            raise AssertionError(f"Unsupported bound type {bt} for variable {t[2]}")
        j = colm[t[2]]
        if bt == "LO":
            lb[j] = float(t[3])
        elif bt == "UP":
            ub[j] = float(t[3])
        elif bt == "FX":
            lb[j] = ub[j] = float(t[3])
        elif bt == "FR":
            lb[j], ub[j] = -np.inf, np.inf
        elif bt == "MI":
            lb[j] = -np.inf
        else:
            ub[j] = np.inf
    if not directions or directions[0] != 'N':
        raise AssertionError(f"First row or cor file is not objective. {''.join(directions)}")
    return spCorType(tok["NAME"][0], directions, row_names, col_names, entries, rhs, lb, ub, colm, rowm)


def read_tim(path) -> spTimType:
    name, periods, section = "", [], ""
    for line in _lines(path):
        t = line.split()
        if line[0] == ' ':
            if section != "PERIODS":
                raise AssertionError("TIM data line outside PERIODS")
            periods.append(spSmpsImplicitPeriod(t[2], spSmpsPosition(t[0], t[1])))
        else:
            section = t[0]
            if section not in ("TIME", "PERIODS", "ENDATA"):
                raise AssertionError(f"unsupported TIM section {section!r}")
            if section == "TIME":
                name = t[1]
    return spTimType(name, periods)


def read_sto(path) -> spStoType:
    sto = spStoType("")
    section, kw = "", []
    for line in _lines(path):
        if not line or line[0] == '*':
            continue
        t = line.split()
        if line[0] == ' ':
            if section != "INDEP":
                continue
            if len(kw) > 1:
                raise ValueError(f"Trailing/unsupported section_keywords {kw}")
            pos = spSmpsPosition(t[0], t[1])
            if kw[0] == "UNIFORM":
                sto.indep[pos] = ("UNIFORM", float(t[2]), float(t[3]))
            elif kw[0] == "NORMAL":
                sto.indep[pos] = ("NORMAL", float(t[2]), float(t[3]))
            elif kw[0] == "DISCRETE":
                if pos not in sto.indep:
                    sto.indep[pos] = ("DISCRETE", [], [])
                sto.indep[pos][1].append(float(t[2]))
                sto.indep[pos][2].append(float(t[3]))
            else:
                raise ValueError(f"Unknown or unsupported section_keywords {kw}")
        else:
            section = t[0]
            if section not in ("STOCH", "INDEP", "ENDATA"):
                raise AssertionError(f"unsupported STO section {section!r}")
            kw = t[1:]
            if section == "STOCH":
                sto.problem_name = kw[0]
    return sto


@dataclass
class spStageProblem:
    """Sparse stage problem: rows (W y + T x) {G,L,E} r, objective q'y (MIN)."""
    last_stage_vars: list
    current_stage_vars: list
    stage_constraints: list
    sense: list
    q: np.ndarray
    r: np.ndarray
    T: tuple           # CSC (colptr, rowval, nzval), m x n1, 0-based int64
    W: tuple           # CSC m x n2
    ylb: np.ndarray
    yub: np.ndarray

    @property
    def shape(self):
        return len(self.stage_constraints), len(self.last_stage_vars), len(self.current_stage_vars)

    def dense_T(self):
        return _csc_dense(self.T, len(self.stage_constraints), len(self.last_stage_vars))

    def dense_W(self):
        return _csc_dense(self.W, len(self.stage_constraints), len(self.current_stage_vars))


def _csc(entries, rows, cols):
    ri = {r: i for i, r in enumerate(rows)}
    colptr = [0]
    rv, nz = [], []
    for c in cols:
        col = sorted((ri[r], v) for (r, cc), v in entries.items() if cc == c and r in ri)
        rv += [i for i, _ in col]
        nz += [v for _, v in col]
        colptr.append(len(rv))
    return (np.array(colptr, dtype=np.int64), np.array(rv, dtype=np.int64), np.array(nz, dtype=np.float64))


def _csc_dense(csc, m, n):
    cp, rv, nz = csc
    A = np.zeros((m, n))
    for j in range(n):
        A[rv[cp[j]:cp[j + 1]], j] = nz[cp[j]:cp[j + 1]]
    return A


def get_smps_stage_template(cor: spCorType, tim: spTimType, stage: int) -> spStageProblem:
    P = tim.periods
    assert 1 <= stage <= len(P)
    start_col = 0 if stage == 1 else cor.col_mapping[P[stage - 2].position.col_name]
    end_col = cor.col_mapping[P[stage].position.col_name] - 1 if stage < len(P) else len(cor.col_names) - 1
    cur_start = cor.col_mapping[P[stage - 1].position.col_name]
    start_row = 1 if stage == 1 else cor.row_mapping[P[stage - 1].position.row_name]
    end_row = cor.row_mapping[P[stage].position.row_name] - 1 if stage < len(P) else len(cor.row_names) - 1
    last = list(range(start_col, cur_start))
    cur = list(range(cur_start, end_col + 1))
    rows = list(range(start_row, end_row + 1))
    # column-sliced entries
    by_col = {}
    for (i, j), v in cor.entries.items():
        by_col.setdefault(j, []).append((i, v))
    rowpos = {r: p for p, r in enumerate(rows)}

    def csc_of(cols):
        colptr, rv, nz = [0], [], []
        for j in cols:
            col = sorted((rowpos[i], v) for i, v in by_col.get(j, []) if i in rowpos)
            rv += [i for i, _ in col]
            nz += [v for _, v in col]
            colptr.append(len(rv))
        return (np.array(colptr, dtype=np.int64), np.array(rv, dtype=np.int64), np.array(nz, dtype=np.float64))

    q = np.array([cor.entries.get((0, j), 0.0) for j in cur])
    return spStageProblem(
        last_stage_vars=[cor.col_names[j] for j in last],
        current_stage_vars=[cor.col_names[j] for j in cur],
        stage_constraints=[cor.row_names[i] for i in rows],
        sense=[cor.directions[i] for i in rows],
        q=q, r=cor.rhs[rows].copy(), T=csc_of(last), W=csc_of(cur),
        ylb=cor.lower_bound[cur].copy(), yub=cor.upper_bound[cur].copy())


def load_smps(directory, name=None):
    """(cor, tim, sto) of an SMPS triple <dir>/<name>.{cor,tim,sto}."""
    name = name or os.path.basename(os.path.normpath(directory))
    base = os.path.join(directory, name)
    return read_cor(base + ".cor"), read_tim(base + ".tim"), read_sto(base + ".sto")


# ---------------------------------------------------------------------- scenarios
def scenario_positions(sp2: spStageProblem, sto: spStoType):
    """Random-element layout for the C ABI: (positions, row[k], col[k] (-1 = RHS)).
    Row/column lookups raise KeyError like delta_coefficients (subprob.jl:112,116)."""
    rowm = {n: i for i, n in enumerate(sp2.stage_constraints)}
    colm = {n: j for j, n in enumerate(sp2.last_stage_vars)}
    positions = list(sto.indep.keys())
    rows = np.array([rowm[p.row_name] for p in positions], dtype=np.int32)
    cols = np.array([-1 if p.col_name in ("RHS", "rhs") else colm[p.col_name] for p in positions], dtype=np.int32)
    return positions, rows, cols


def sample_values(sto: spStoType, N: int, rng: np.random.Generator, positions=None) -> np.ndarray:
    """N i.i.d. draws of every independent element (rand(sto), smps_sto.jl:140-149):
    N x k values in `positions` order.  NORMAL uses sqrt(variance) (smps_sto.jl:122-125)."""
    positions = positions if positions is not None else list(sto.indep.keys())
    out = np.empty((N, len(positions)))
    for e, p in enumerate(positions):
        d = sto.indep[p]
        if d[0] == "DISCRETE":
            vals = np.asarray(d[1], dtype=np.float64)
            cdf = np.cumsum(np.asarray(d[2], dtype=np.float64))
            u = rng.random(N) * cdf[-1]
            out[:, e] = vals[np.minimum(np.searchsorted(cdf, u, side="right"), len(vals) - 1)]
        elif d[0] == "NORMAL":
            out[:, e] = rng.normal(d[1], np.sqrt(d[2]), size=N)
        else:
            out[:, e] = rng.uniform(d[1], d[2], size=N)
    return out


def mean_values(sto: spStoType, positions=None) -> np.ndarray:
    positions = positions if positions is not None else list(sto.indep.keys())
    out = []
    for p in positions:
        d = sto.indep[p]
        if d[0] == "DISCRETE":
            out.append(float(np.dot(d[1], d[2]) / np.sum(d[2])))
        elif d[0] == "NORMAL":
            out.append(d[1])
        else:
            out.append(0.5 * (d[1] + d[2]))
    return np.array(out)

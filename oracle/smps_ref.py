"""SMPS restatement (oracle; TEST INFRASTRUCTURE ONLY -- see oracle/__init__.py).

Line-by-line restatement of the reference's SMPS reader and stage split:
  * ``tokenize_cor``      <- src/smps/smps_cor.jl:26-58   (_tokenize_cor)
  * ``parse_row_tokens``  <- src/smps/smps_cor.jl:63-67
  * ``parse_unique_columns`` <- src/smps/smps_cor.jl:72-75
  * ``parse_column_to_matrix`` <- src/smps/smps_cor.jl:81-101
  * ``parse_rhs``         <- src/smps/smps_cor.jl:106-116
  * ``parse_bounds``      <- src/smps/smps_cor.jl:124-155
  * ``read_cor``          <- src/smps/smps_cor.jl:160-194
  * ``read_tim``          <- src/smps/smps_tim.jl:30-64
  * ``read_sto``          <- src/smps/smps_sto.jl:41-110
  * ``stage_template``    <- src/smps/smps_prob.jl:14-102 (get_smps_stage_template)

Dense numpy storage is used on purpose (instances are small; clarity over speed).
"""
from __future__ import annotations

from dataclasses import dataclass, field
import numpy as np


@dataclass
class Cor:
    problem_name: str
    directions: list
    row_names: list
    col_names: list
    matrix: np.ndarray          # dense (nrows x ncols)
    rhs: np.ndarray
    lower_bound: np.ndarray
    upper_bound: np.ndarray
    col_mapping: dict
    row_mapping: dict


@dataclass
class Tim:
    problem_name: str
    periods: list               # [(period_name, col_name, row_name)]


@dataclass
class Sto:
    problem_name: str
    # insertion-ordered: position (col_name,row_name) -> ("DISCRETE", values, probs)
    #                   | ("NORMAL", mean, variance) | ("UNIFORM", a, b)
    indep: dict = field(default_factory=dict)


def _julia_split(line: str):
    return line.split()


def tokenize_cor(lines):
    """smps_cor.jl:26-58.  Lines that are empty or start with '*' are dropped; a line
    whose first character is not ' ' is a section header (asserted supported)."""
    supported = ["NAME", "ROWS", "COLUMNS", "RHS", "BOUNDS", "ENDATA"]
    tokens = {s: [] for s in supported}
    lines = [s for s in lines if len(s) > 0 and s[0] != '*']
    section = ""
    for line in lines:
        token = _julia_split(line)
        if line[0] != ' ':
            section = token[0]
            assert section in supported, f"unsupported section {section}"
            if token[0] == "NAME":
                tokens["NAME"].append(token[1])      # smps_cor.jl:48-50 (throws if absent)
        else:
            tokens[section].append(token)
    return tokens


def parse_row_tokens(tokens):
    return [t[0][0] for t in tokens], [t[1] for t in tokens]


def parse_unique_columns(tokens):
    seen, out = set(), []
    for t in tokens:
        if t[0] not in seen:
            seen.add(t[0])
            out.append(t[0])
    return out


def parse_column_to_matrix(tokens, row_names, col_names):
    colm = {c: i for i, c in enumerate(col_names)}
    rowm = {r: i for i, r in enumerate(row_names)}
    M = np.zeros((len(row_names), len(col_names)))
    for t in tokens:
        j = colm[t[0]]
        rest = t[1:]
        for a in range(0, len(rest), 2):
            M[rowm[rest[a]], j] = float(rest[a + 1])
    return M


def parse_rhs(tokens, row_names):
    rowm = {r: i for i, r in enumerate(row_names)}
    rhs = np.zeros(len(row_names))
    for t in tokens:
        rest = t[1:]
        for a in range(0, len(rest), 2):
            rhs[rowm[rest[a]]] = float(rest[a + 1])
    return rhs


def parse_bounds(tokens, col_names):
    supported = ["LO", "UP", "FX", "FR", "MI", "PL"]
    colm = {c: i for i, c in enumerate(col_names)}
    lb = np.zeros(len(col_names))
    ub = np.full(len(col_names), np.inf)
    for t in tokens:
        bt = t[0]
        assert bt in supported, f"Unsupported bound type {bt}"
        j = colm[t[2]]
        if bt == "LO":
            lb[j] = float(t[3])
        elif bt == "UP":
            ub[j] = float(t[3])
        elif bt == "FX":
            lb[j] = float(t[3]); ub[j] = float(t[3])
        elif bt == "FR":
            lb[j] = -np.inf; ub[j] = np.inf
        elif bt == "MI":
            lb[j] = -np.inf
        elif bt == "PL":
            ub[j] = np.inf
    return lb, ub


def _readlines(path):
    with open(path, "r", encoding="latin-1") as f:
        return f.read().splitlines()


def read_cor(path) -> Cor:
    tok = tokenize_cor(_readlines(path))
    name = tok["NAME"][0]
    dirs, rows = parse_row_tokens(tok["ROWS"])
    cols = parse_unique_columns(tok["COLUMNS"])
    M = parse_column_to_matrix(tok["COLUMNS"], rows, cols)
    rhs = parse_rhs(tok["RHS"], rows)
    lb, ub = parse_bounds(tok["BOUNDS"], cols)
    assert dirs[0] == 'N', "First row or cor file is not objective."   # smps_cor.jl:178
    return Cor(name, dirs, rows, cols, M, rhs, lb, ub,
               {c: i for i, c in enumerate(cols)}, {r: i for i, r in enumerate(rows)})


def read_tim(path) -> Tim:
    """smps_tim.jl:30-64 (no comment filtering in the reference)."""
    section, name, periods = "", "", []
    for line in _readlines(path):
        token = _julia_split(line)
        if line[0] == ' ':
            assert section == "PERIODS"
            periods.append((token[2], token[0], token[1]))
        else:
            section = token[0]
            assert section in ["TIME", "PERIODS", "ENDATA"]
            if section == "TIME":
                name = token[1]
    return Tim(name, periods)


def read_sto(path) -> Sto:
    """smps_sto.jl:41-110: INDEP DISCRETE / NORMAL(mean, variance) / UNIFORM(a, b)."""
    lines = [s for s in _readlines(path) if len(s) > 0 and s[0] != '*']
    sto = Sto("")
    section, kw = "", []
    for line in lines:
        token = _julia_split(line)
        if line[0] == ' ':
            if section == "INDEP":
                pos = (token[0], token[1])
                if len(kw) > 1:
                    raise ValueError(f"Trailing/unsupported section_keywords {kw}")
                if kw[0] == "UNIFORM":
                    sto.indep[pos] = ("UNIFORM", float(token[2]), float(token[3]))
                elif kw[0] == "NORMAL":
                    sto.indep[pos] = ("NORMAL", float(token[2]), float(token[3]))
                elif kw[0] == "DISCRETE":
                    if pos not in sto.indep:
                        sto.indep[pos] = ("DISCRETE", [], [])
                    sto.indep[pos][1].append(float(token[2]))
                    sto.indep[pos][2].append(float(token[3]))
                else:
                    raise ValueError(f"Unknown or unsupported section_keywords {kw}")
        else:
            section = token[0]
            assert section in ["STOCH", "INDEP", "ENDATA"]
            kw = token[1:]
            if section == "STOCH":
                sto.problem_name = kw[0]
    return sto


@dataclass
class StageProblem:
    """Dense restatement of spStageProblem (src/prob.jl:10-15) for the oracle."""
    last_names: list
    cur_names: list
    row_names: list
    senses: list                  # 'G' | 'L' | 'E' per stage row
    q: np.ndarray                 # objective over current-stage vars
    T: np.ndarray                 # rows x last-stage vars
    W: np.ndarray                 # rows x current-stage vars
    r: np.ndarray                 # rhs
    cur_lb: np.ndarray
    cur_ub: np.ndarray


def stage_template(cor: Cor, tim: Tim, stage: int) -> StageProblem:
    """smps_prob.jl:14-102 (stage is 1-based as in the reference)."""
    P = tim.periods
    assert 1 <= stage <= len(P)
    start_col = 0 if stage == 1 else cor.col_mapping[P[stage - 2][1]]
    end_col = (cor.col_mapping[P[stage][1]] - 1) if stage < len(P) else len(cor.col_names) - 1
    cur_start = cor.col_mapping[P[stage - 1][1]]
    start_row = 1 if stage == 1 else cor.row_mapping[P[stage - 1][2]]
    end_row = (cor.row_mapping[P[stage][2]] - 1) if stage < len(P) else len(cor.row_names) - 1
    last = list(range(start_col, cur_start))
    cur = list(range(cur_start, end_col + 1))
    rows = list(range(start_row, end_row + 1))
    M = cor.matrix
    return StageProblem(
        last_names=[cor.col_names[j] for j in last],
        cur_names=[cor.col_names[j] for j in cur],
        row_names=[cor.row_names[i] for i in rows],
        senses=[cor.directions[i] for i in rows],
        q=M[0, cur].copy(),
        T=M[np.ix_(rows, last)].copy() if last else np.zeros((len(rows), 0)),
        W=M[np.ix_(rows, cur)].copy(),
        r=cor.rhs[rows].copy(),
        cur_lb=cor.lower_bound[cur].copy(),
        cur_ub=cor.upper_bound[cur].copy(),
    )


def load_instance(dirpath, name):
    import os
    cor = read_cor(os.path.join(dirpath, name + ".cor"))
    tim = read_tim(os.path.join(dirpath, name + ".tim"))
    sto = read_sto(os.path.join(dirpath, name + ".sto"))
    return cor, tim, sto

"""Shared test helpers: instance loading through both the product loader (sqlp_amd.smps)
and the oracle restatement, EV first-stage x, seeded scenario samples."""
from __future__ import annotations

import functools
import os

import numpy as np

from oracle import lp_highs, smps_ref
from sqlp_amd import smps

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DATA = os.path.join(ROOT, "data", "smps")
INSTANCES = ["lands", "newsvendor", "transship", "ssn", "storm"]


@functools.lru_cache(maxsize=None)
def load(name):
    d = os.path.join(DATA, name)
    cor, tim, sto = smps.load_smps(d, name)
    sp2 = smps.get_smps_stage_template(cor, tim, 2)
    ocor, otim, osto = smps_ref.load_instance(d, name)
    osp1 = smps_ref.stage_template(ocor, otim, 1)
    osp2 = smps_ref.stage_template(ocor, otim, 2)
    return dict(cor=cor, tim=tim, sto=sto, sp2=sp2, osp1=osp1, osp2=osp2, osto=osto)


@functools.lru_cache(maxsize=None)
def x_ev(name):
    I = load(name)
    r2 = lp_highs.sto_mean_rhs(I["osp2"], I["osto"])
    _, x = lp_highs.solve_ev(I["osp1"], I["osp2"], r2)
    return np.asarray(x)


def sample(name, N, seed):
    I = load(name)
    return smps.sample_values(I["sto"], N, np.random.default_rng(seed))


def rhs_of(name, x, values):
    """Full stage-2 rhs b = r_w - T x for RHS-only instances (oracle side)."""
    I = load(name)
    sp = I["osp2"]
    pos, rows, cols = smps.scenario_positions(I["sp2"], I["sto"])
    assert (cols < 0).all()
    b = np.tile(sp.r - sp.T @ x, (values.shape[0], 1))
    b[:, rows] += values - sp.r[rows]
    return b

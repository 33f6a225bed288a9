"""Host plumbing on CPU: the product SMPS loader against the oracle restatement and the
reference's parser KATs; the C ABI library exports every symbol of include/twosd_hip.h."""
import ctypes
import os
import re

import numpy as np
import pytest

from sqlp_amd import smps
from tests import instances as I

ROOT = I.ROOT


@pytest.mark.parametrize("name", I.INSTANCES + ["baa99-20"])
def test_product_loader_matches_oracle(name):
    inst = I.load(name) if name in I.INSTANCES else None
    d = os.path.join(I.DATA, name)
    cor, tim, sto = smps.load_smps(d, name)
    sp2 = smps.get_smps_stage_template(cor, tim, 2)
    from oracle import smps_ref
    ocor, otim, osto = smps_ref.load_instance(d, name)
    osp2 = smps_ref.stage_template(ocor, otim, 2)
    assert sp2.stage_constraints == osp2.row_names
    assert sp2.current_stage_vars == osp2.cur_names and sp2.last_stage_vars == osp2.last_names
    assert sp2.sense == osp2.senses
    np.testing.assert_array_equal(sp2.dense_W(), osp2.W)
    np.testing.assert_array_equal(sp2.dense_T(), osp2.T)
    np.testing.assert_array_equal(sp2.q, osp2.q)
    np.testing.assert_array_equal(sp2.r, osp2.r)
    assert list(sto.indep.keys()) == [smps.spSmpsPosition(*p) for p in osto.indep.keys()]


def test_product_loader_kats():
    # test/smps_tests.jl:36-58, 71 on the product loader
    cor, tim, sto = smps.load_smps(os.path.join(I.DATA, "lands"), "lands")
    assert "".join(cor.directions) == "NGLLLLLGGG" and len(cor.entries) == 52
    assert tim.periods[1].position == smps.spSmpsPosition("Y11", "S2C1")
    sp1 = smps.get_smps_stage_template(cor, tim, 1)
    sp2 = smps.get_smps_stage_template(cor, tim, 2)
    assert sp1.shape == (2, 0, 4) and sp2.shape == (7, 4, 12)
    pos = smps.spSmpsPosition("RHS", "S2C5")
    assert sto.indep[pos][1] == [3.0, 5.0, 7.0]
    v = smps.sample_values(sto, 1000, np.random.default_rng(1234))
    assert set(np.unique(v)) <= {3.0, 5.0, 7.0}                     # smps_tests.jl:63,66
    freq = np.array([(v == t).mean() for t in (3.0, 5.0, 7.0)])
    assert np.allclose(freq, [0.3, 0.4, 0.3], atol=0.05)


def test_sampler_distributions():
    cor, tim, sto = smps.load_smps(os.path.join(I.DATA, "transship"), "transship")
    v = smps.sample_values(sto, 200000, np.random.default_rng(5))
    means = np.array([d[1] for d in sto.indep.values()])
    stds = np.sqrt([d[2] for d in sto.indep.values()])          # NORMAL(mean, variance)
    assert np.allclose(v.mean(0), means, atol=0.05 * stds.max())
    assert np.allclose(v.std(0), stds, rtol=0.02)


def test_positions_keyerror():
    # delta_coefficients raises KeyError for a non-first-stage column (subprob.jl:116)
    cor, tim, sto = smps.load_smps(os.path.join(I.DATA, "lands"), "lands")
    sp2 = smps.get_smps_stage_template(cor, tim, 2)
    sto.indep[smps.spSmpsPosition("Y11", "S2C5")] = ("DISCRETE", [1.0], [1.0])
    with pytest.raises(KeyError):
        smps.scenario_positions(sp2, sto)


def test_missing_name_record_raises():
    # smps_cor.jl:48-50: NAME without a token is a BoundsError in the reference
    with pytest.raises(IndexError):
        smps.read_cor(os.path.join(I.DATA, "newsvendor", "newsvendor.mps"))


def _header_symbols():
    with open(os.path.join(ROOT, "include", "twosd_hip.h")) as f:
        text = f.read()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\s*\*?\s*(twosd_\w+)\s*\(", text, re.M)))


def test_library_exports_every_header_symbol():
    from sqlp_amd import _lib
    syms = _header_symbols()
    assert len(syms) >= 25
    lib = ctypes.CDLL(_lib.LIB_PATH)
    missing = [s for s in syms if not hasattr(lib, s)]
    assert not missing, missing
    # and the ctypes table binds exactly the header
    assert sorted(n for n, _, _ in _lib.SIGNATURES) == syms


def test_library_version_without_gpu():
    from sqlp_amd import _lib
    assert b"gfx950" in _lib.load().twosd_version()

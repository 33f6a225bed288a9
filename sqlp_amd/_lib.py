"""ctypes binding of libtwosd_hip.so (the C ABI declared in include/twosd_hip.h).

The shared library is built in-tree (``sqlp_amd/libtwosd_hip.so``, see
``__graft_entry__.build()``).  There is no CPU fallback: if the library is missing or
cannot be loaded, every call raises.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# TWOSD_LIB=<variant> selects libtwosd_hip_<variant>.so (e.g. "stamps": the phase-stamp
# diagnostic build, never used for timing claims; tuning variants during development)
LIB_PATH = os.path.join(_HERE, f"libtwosd_hip_{os.environ['TWOSD_LIB']}.so" if os.environ.get("TWOSD_LIB")
                        else "libtwosd_hip.so")

TWOSD_OK = 0
ERRORS = {-1: "TWOSD_E_ARG", -2: "TWOSD_E_DEVICE", -3: "TWOSD_E_STATE", -4: "TWOSD_E_LP",
          -5: "TWOSD_E_UNSUPPORTED"}
LP_OPTIMAL, LP_INFEASIBLE, LP_ITER_LIMIT, LP_NUMERIC = 0, 1, 2, 3

# (name, restype, argtypes) for every symbol declared in include/twosd_hip.h
P = C.c_void_p
I = C.c_int
D = C.c_double
SIGNATURES = [
    ("twosd_last_error", C.c_char_p, []),
    ("twosd_version", C.c_char_p, []),
    ("twosd_create", I, [I, P]),
    ("twosd_destroy", I, [P]),
    ("twosd_set_template", I, [P, I, I, I, P, P, P, P, P, P, P, P, P, P, P, I]),
    ("twosd_set_random_positions", I, [P, I, P, P, I]),
    ("twosd_compute_basis", I, [P, P, P]),
    ("twosd_set_basis", I, [P, P]),
    ("twosd_get_basis", I, [P, P]),
    ("twosd_pool_add_basis", I, [P, P, P]),
    ("twosd_pool_build", I, [P, I, P, I, I, I, P]),
    ("twosd_pool_build_candidates", I, [P, I, P, I, I, I, I]),
    ("twosd_pool_refresh", I, [P, I, P, I, I, I, P]),
    ("twosd_last_refresh_ms", I, [P, P]),
    ("twosd_pool_size", I, [P, P]),
    ("twosd_pool_get", I, [P, I, P]),
    ("twosd_last_pool_picks", I, [P, I, P]),
    ("twosd_invalidate_x", I, [P]),
    ("twosd_epigraph_create", I, [P, P]),
    ("twosd_add_scenarios", I, [P, I, I, P, P]),
    ("twosd_epigraph_info", I, [P, I, P, P]),
    ("twosd_set_distributions", I, [P, I, P, P, P, P, P, P]),
    ("twosd_add_sampled_scenarios", I, [P, I, I, C.c_uint64, C.c_uint64, P]),
    ("twosd_get_scenarios", I, [P, I, I, I, P]),
    ("twosd_evaluate_sampled", I, [P, P, C.c_int64, C.c_int64, C.c_int64, C.c_uint64, P]),
    ("twosd_solve_batch", I, [P, I, P, I, I, P, P, P, P]),
    ("twosd_solve_values", I, [P, P, I, P, P, P, P, P]),
    ("twosd_dvs_push", I, [P, I, P, P, P]),
    ("twosd_dvs_size", I, [P, P]),
    ("twosd_dvs_get", I, [P, I, I, P]),
    ("twosd_dvs_clear", I, [P]),
    ("twosd_dvs_truncate", I, [P, I]),
    ("twosd_dvs_fingerprint", I, [P, P]),
    ("twosd_solve_push", I, [P, I, P, I, I, P, P, P]),
    ("twosd_last_push_reps", I, [P, P]),
    ("twosd_last_push_mode", I, [P, P]),
    ("twosd_build_cut", I, [P, I, P, D, P, P, P, P, P]),
    ("twosd_cut_partial_len", I, [P, P, P]),
    ("twosd_cut_partial", I, [P, I, P, D, D, P, P, P, P]),
    ("twosd_cut_finalize", I, [P, P, P, P, P, P]),
    ("twosd_last_timings", I, [P, P]),
    ("twosd_last_lp_stats", I, [P, P, P]),
    ("twosd_last_lp_eta_entries", I, [P, P, P]),
    ("twosd_last_lp_ops", I, [P, P, P]),
    ("twosd_debug_stamps", I, [P, P, I]),
    ("twosd_last_lp_iters", I, [P, I, P, P]),
    ("twosd_set_refresh_kcap", I, [P, I]),
    ("twosd_refresh_train", I, [P, I, P, I, I, P, P, P]),
    ("twosd_refresh_train_ex", I, [P, I, P, I, I, I, P, P, P, P]),
    ("twosd_refresh_cap_stats", I, [P, P, P]),
    ("twosd_training_cap", I, [P, C.c_int64, C.c_int64, P]),
    ("twosd_cut_stats", I, [P, P]),
    ("twosd_cut_pass", I, [P, P, P]),
    ("twosd_select_refresh_bases", I, [P, P, P, P, I, I, P, P, P]),
    ("twosd_last_objective", I, [P, P, P]),
    ("twosd_refresh_train_bases", I, [P, P, P, P]),
    ("twosd_refresh_build_local", I, [P, I, P, P]),
    ("twosd_refresh_pack", I, [P, P]),
    ("twosd_refresh_assemble", I, [P, I, P, C.c_int64, I, P, P, P, P]),
    ("twosd_pool_candidate_picks", I, [P, I, P, I, I, I, P, P]),
    ("twosd_pool_set_candidates", I, [P, I, I, I, P, P]),
]

_lib = None


class TwoSDError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"{ERRORS.get(code, code)}: {msg}")
        self.code = code


def load():
    """Load the in-tree HIP library (raises if it has not been built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} not built: run __graft_entry__.build() (make -C sqlp_amd/csrc)")
        lib = C.CDLL(LIB_PATH)
        for name, res, args in SIGNATURES:
            f = getattr(lib, name)
            f.restype = res
            f.argtypes = args
        _lib = lib
    return _lib


def check(rc):
    if rc != TWOSD_OK:
        raise TwoSDError(rc, load().twosd_last_error().decode())
    return rc


def ptr(a):
    """Pointer to a contiguous numpy array (or None)."""
    if a is None:
        return None
    return a.ctypes.data_as(C.c_void_p)

"""sqlp_amd -- MI355X-native TwoSD scenario-subproblem + cut-generation hot path.

The compute lives in libtwosd_hip.so (hand-written HIP for gfx950, C ABI in
include/twosd_hip.h); ``sqlp_amd.twosd`` is the host-side mirror of the reference's
TwoSD API for that path and ``sqlp_amd.smps`` the SMPS loader that feeds it.
"""
from . import smps  # noqa: F401

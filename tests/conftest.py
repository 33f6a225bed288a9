import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

DATA = os.path.join(ROOT, "data", "smps")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libtwosd_hip.so)")
    config.addinivalue_line("markers", "slow: long CPU test")


@pytest.fixture(scope="session")
def data_dir():
    return DATA


def pytest_collection_modifyitems(config, items):
    # GPU sessions: bring up torch's HIP runtime before libtwosd_hip.so touches the device,
    # as bench.py does (tests that hand torch device tensors to the library need torch's
    # runtime; initialising it after the library's has been seen to find no devices)
    if "not gpu" in (config.getoption("-m") or ""):
        return
    if any(item.get_closest_marker("gpu") for item in items):
        try:
            import torch
            if torch.cuda.is_available():
                torch.cuda.init()
        except Exception:
            pass

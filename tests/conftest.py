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

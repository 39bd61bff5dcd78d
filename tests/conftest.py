import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run through gpurun)")
    config.addinivalue_line("markers", "dist: spawns multiple processes (gloo on CPU)")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(autouse=True)
def _reset_parallel_state():
    yield
    try:
        from mxtrain.parallel import state as pstate
        pstate._STATE = None
    except Exception:
        pass

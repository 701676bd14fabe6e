import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device); run with -m gpu")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(scope="session")
def golden():
    import _golden
    return _golden.load_vectors()


@pytest.fixture(scope="session")
def engine():
    from firedancer_amd import ed25519
    eng = ed25519.Engine(device=0, batch_max=1 << 16, blob_max=(1 << 16) * 300)
    yield eng
    eng.close()

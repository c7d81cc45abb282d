import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "oracle"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libsng_hip.so)")


@pytest.fixture(scope="session")
def synthetic_model():
    from synerfgine_amd import synthetic
    return synthetic.lego_like(seed=1337)


@pytest.fixture(scope="session")
def oracle_lib():
    import oracle as O
    O.lib()
    return O

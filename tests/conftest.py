import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(REPO, "tests", "golden")
if REPO not in sys.path:
    sys.path.insert(0, REPO)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device)")


def golden(name):
    return np.load(os.path.join(GOLDEN, f"golden_{name}.npz"), allow_pickle=False)


@pytest.fixture(scope="session")
def score_sd():
    from genpose2_amd import weights
    return weights.synthetic_state_dict("score", seed=0)


@pytest.fixture(scope="session")
def energy_sd():
    from genpose2_amd import weights
    return weights.synthetic_state_dict("energy", seed=0)


@pytest.fixture(scope="session")
def scale_sd():
    from genpose2_amd import weights
    return weights.synthetic_state_dict("scale", seed=0)

import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libdse on the device)")
    config.addinivalue_line("markers", "slow: longer CPU test")


@pytest.fixture(scope="session")
def golden():
    """Loader for the committed fixtures (numpy/JSON only; nothing is unpickled)."""
    import json

    def load(name):
        path = os.path.join(GOLDEN, name)
        if name.endswith(".json"):
            with open(path) as f:
                return json.load(f)
        return np.load(path, allow_pickle=False)
    return load


@pytest.fixture(scope="session")
def engine():
    """One device context for the whole GPU session (tests clear it between uses)."""
    from quantumsimulations_amd.engine import Engine, device_count
    if device_count() < 1:
        pytest.fail("GPU test selected but no HIP device is visible")
    eng = Engine(0)
    yield eng
    eng.close()


def csr_from(npz, key):
    import scipy.sparse as sp
    data, ind, ptr = npz[f"{key}_data"], npz[f"{key}_indices"], npz[f"{key}_indptr"]
    n = len(ptr) - 1
    return sp.csr_matrix((data, ind, ptr), shape=(n, n))

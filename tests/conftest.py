import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "ds-gan_amd")
for p in (REPO, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libdsgan_hip.so)")
    config.addinivalue_line("markers", "slow: long-running")


def gpu_available():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope="session")
def golden():
    import numpy as np
    return np.load(os.path.join(REPO, "tests", "golden", "golden_v1.npz"))


@pytest.fixture(scope="session")
def golden_v3():
    import numpy as np
    return np.load(os.path.join(REPO, "tests", "golden", "golden_v3.npz"))


@pytest.fixture(scope="session")
def golden_v4():
    import numpy as np
    return np.load(os.path.join(REPO, "tests", "golden", "golden_v4.npz"))

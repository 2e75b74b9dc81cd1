import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "gripper-mujoco_amd")
for p in (PKG, os.path.join(REPO, "tests"), REPO):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C ABI)")
    config.addinivalue_line("markers", "slow: long-running test")


@pytest.fixture(scope="session")
def gm():
    import gmx
    from gmx.build import build
    if not os.path.exists(gmx.LIB_PATH):
        build()
    gmx.load_library()
    return gmx


@pytest.fixture(scope="session")
def model(gm):
    return gm.ModelBlob()


def gpu_available():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False

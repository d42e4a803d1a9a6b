import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

WISDM_CANDIDATES = [
    os.environ.get("HAR_WISDM_CSV", ""),
    os.path.join(ROOT, "data", "wisdm_data.csv"),
    # WISDM v1.1 transformed table (the reference's dataset, Main/wisdm_main_ver_0.0/data/wisdm_data.csv),
    # vendored so the GPU box — where /root/reference does not exist — runs the WISDM tests too
    os.path.join(ROOT, "tests", "data", "wisdm_data.csv"),
    "/root/reference/Main/wisdm_main_ver_0.0/data/wisdm_data.csv",
]


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels)")
    config.addinivalue_line("markers", "slow: longer CPU tests")


def wisdm_path():
    for p in WISDM_CANDIDATES:
        if p and os.path.exists(p):
            return p
    return None


@pytest.fixture(scope="session")
def wisdm_csv():
    p = wisdm_path()
    if p is None:
        pytest.skip("WISDM CSV not available (set HAR_WISDM_CSV)")
    return p


@pytest.fixture(scope="session")
def cuda():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")

import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI)")


def gpu_available() -> bool:
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope="session")
def cuda():
    import torch
    if not torch.cuda.is_available():
        # -m gpu runs only on the MI355X box: a missing GPU there is a failure, not a skip
        pytest.fail("GPU test requested but torch.cuda.is_available() is False")
    return torch.device("cuda:0")


@pytest.fixture(params=["pipe", "fused"])
def back(request, monkeypatch):
    """Both back-end kernels: the wave pipeline (rx_back, small batches) and the fused
    one-wave-per-64-channels kernel (rx_back_fused, large batches), forced per handle."""
    monkeypatch.setenv("UHSDR_BACK_FUSED", "1" if request.param == "fused" else "0")
    return request.param

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


SCHEDULES = {"pipe": 1, "fused": 2, "chain": 3}   # uhsdr_rx_set_schedule values


@pytest.fixture(params=["pipe", "fused", "chain"])
def back(request, monkeypatch):
    """Every kernel schedule of a call: the back-end wave pipeline (rx_back, small batches), the
    fused one-wave-per-64-channels back end (rx_back_fused), and the one-kernel rx_chain (front
    passes + fused back end per wave, large batches), forced on every RxChain the test makes.
    rx_chain covers the SSB / CW / DIGI mono paths; elsewhere the handles keep the AUTO choice."""
    from uhsdr_amd import rx
    monkeypatch.setattr(rx, "DEFAULT_SCHEDULE", SCHEDULES[request.param])
    return request.param

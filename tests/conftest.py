import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 GPU (runs on the MI355X box)")
    config.addinivalue_line("markers", "slow: long-running parity sweep")


import pytest  # noqa: E402


@pytest.fixture(scope="session", autouse=True)
def _torch_hip_first(request):
    """PyTorch's wheel bundles its own HIP/HSA runtime next to the /opt/rocm one liborbfe.so
    links.  When both live in one process, torch's runtime must initialise first (as bench.py
    does); otherwise torch reports "No HIP GPUs are available".  Only for sessions that run GPU
    tests on a machine with a GPU."""
    if any(item.get_closest_marker("gpu") for item in request.session.items):
        import torch
        if torch.cuda.is_available():
            torch.cuda.init()
            torch.zeros(1, device="cuda:0")
    yield

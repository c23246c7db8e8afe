import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "celestia-app_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs through libcda on the device)")


@pytest.fixture(scope="session", autouse=True)
def _torch_hip_first(request):
    """PyTorch ships its own HIP / HSA runtime (torch/lib) while libcda links /opt/rocm's; with both in one process
    torch's must initialise first, or torch.cuda reports "No HIP GPUs are available" (libcda works either way).
    A Go node has no torch: this concerns the Python tests and tools only."""
    if any(item.get_closest_marker("gpu") for item in request.session.items):
        import torch
        if torch.cuda.is_available():
            torch.cuda.init()
    yield


@pytest.fixture(scope="session")
def ctx():
    import cda
    c = cda.Context(0)
    yield c
    c.close()

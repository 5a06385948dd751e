import os
import sys

import pytest

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU; run with -m gpu")


@pytest.fixture(autouse=True)
def _torch_hip_first(request):
    """GPU tests: initialise torch's bundled HIP runtime before the library's /opt/rocm one
    (the order bench.py uses); the other order left torch without a device on one box."""
    if request.node.get_closest_marker("gpu") is not None:
        import torch
        torch.cuda.init()
    yield

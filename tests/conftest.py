import os
import sys

import pytest

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU; run with -m gpu")


@pytest.fixture(scope="session", autouse=True)
def _torch_hip_first(request):
    """GPU runs: initialise torch's bundled HIP runtime before the library's /opt/rocm one (the
    order bench.py uses).  The other order leaves torch without a device ("No HIP GPUs are
    available"), so this is session-scoped: it must precede module-scoped engine fixtures."""
    if any(item.get_closest_marker("gpu") is not None for item in request.session.items):
        import torch
        try:
            torch.cuda.init()
        except RuntimeError:  # no GPU here (a CPU run that selected GPU tests): they fail on their own
            pass
    yield

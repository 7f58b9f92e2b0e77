import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run on the GPU box with -m gpu)")
    config.addinivalue_line("markers", "slow: longer CPU test")


def _gpu_run(config):
    """True when the session selects the GPU tests (-m gpu): there a missing device is a failure."""
    expr = (config.getoption("markexpr", "") or "").replace(" ", "")
    return "gpu" in expr and "notgpu" not in expr


@pytest.fixture(scope="session")
def cuda(request):
    import torch
    if not torch.cuda.is_available():
        if _gpu_run(request.config):
            pytest.fail("-m gpu selected but torch.cuda.is_available() is False: the GPU runtime is broken or no "
                        "device is visible (a GPU run must not turn into skips)")
        pytest.skip("no GPU")
    return torch.device("cuda", 0)

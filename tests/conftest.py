import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device)")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(autouse=True)
def _fresh_default_graph():
    from tensorframes_amd.graph import dsl
    dsl.reset_default_graph()
    yield


def gpu_available():
    import torch
    return torch.cuda.is_available()


@pytest.fixture(params=["cpu", pytest.param("cuda", marks=pytest.mark.gpu)])
def on_device(request):
    """Runs a test once on the host executor and once (gpu-marked) with every
    op forced onto the GPU (`Config.device = "cuda"`): the reference's
    acceptance corpus then executes the HIP kernels."""
    import torch
    from tensorframes_amd.config import config
    if request.param == "cuda" and not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    old = config.device
    config.device = request.param
    yield request.param
    config.device = old

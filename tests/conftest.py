import os
import sys

import pytest

_REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(_REPO, "tests"))
sys.path.insert(0, os.path.join(_REPO, "metal-flash-attention-plus_amd", "python"))
sys.path.insert(0, _REPO)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libmfa_amd.so on cuda:0)")
    config.addinivalue_line("markers", "slow: long-running parity case")


@pytest.fixture(scope="session")
def gpu():
    """The GPU tests must run on the HIP path: fail loudly when there is no device."""
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU test selected but torch.cuda is not available (no MI355X visible)")
    return torch.device("cuda:0")

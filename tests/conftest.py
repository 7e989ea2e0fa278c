import os
import sys

import pytest

# The tests A/B the library's development switches (MFA_FWD_SHARE, MFA_KV_REGS, ...), which the
# library reads only in a process started with MFA_DEV=1 (mfa_launch.h dev_env): set it before
# the library is loaded.  tests/test_dev_gate.py checks a process without it.
os.environ.setdefault("MFA_DEV", "1")

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

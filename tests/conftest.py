import sys
from pathlib import Path

import pytest

REPO = Path(__file__).resolve().parent.parent
if str(REPO) not in sys.path:
    sys.path.insert(0, str(REPO))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")


@pytest.fixture(scope="session")
def golden():
    from tests.golden_io import load_golden

    return load_golden()


@pytest.fixture(scope="session")
def hip_device():
    import torch

    from distributed_learning_simulation_lib_amd import _native

    _native.load()  # fails loudly if the HIP library is missing
    assert torch.cuda.is_available(), "GPU tests need a visible MI355X"
    return torch.device("cuda", 0)

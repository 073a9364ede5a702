import pathlib
import sys

import numpy as np
import pytest

ROOT = pathlib.Path(__file__).resolve().parents[1]
if str(ROOT) not in sys.path:
    sys.path.insert(0, str(ROOT))

GOLDEN = ROOT / "tests" / "golden" / "golden.npz"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")


@pytest.fixture(scope="session")
def golden():
    with np.load(GOLDEN, allow_pickle=False) as g:
        return {k: g[k] for k in g.files}


@pytest.fixture(scope="session")
def tw():
    import tuplewise
    return tuplewise


@pytest.fixture(scope="session")
def gpu(tw):
    """Skip-free GPU guard: a gpu-marked test on a machine without a device must FAIL."""
    import torch
    assert torch.cuda.is_available(), "gpu test run without a HIP device"
    return torch.device("cuda", 0)

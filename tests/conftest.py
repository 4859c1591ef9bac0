import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI)")
    config.addinivalue_line("markers", "slow: long CPU run (opt-in with -m slow)")


def golden(name):
    return np.load(os.path.join(GOLDEN, name + ".npz"))


@pytest.fixture(scope="session")
def oracle():
    from oracle import oracle as O
    return O


@pytest.fixture(scope="session")
def gpu():
    """The product path on cuda:0; a GPU test must never fall back to anything else."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import pyrmt_amd
    return pyrmt_amd

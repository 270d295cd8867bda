"""Shared test plumbing: import paths, golden-fixture loader, GPU gating."""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "information-retrieval-with-contrastive-learning_amd")
GOLDEN = os.path.join(ROOT, "tests", "golden")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 (MI355X) HIP device")
    config.addinivalue_line("markers", "slow: longer CPU tests")


def load_golden(name):
    with np.load(os.path.join(GOLDEN, name), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


@pytest.fixture(scope="session")
def gpu():
    """The HIP library + cuda:0, or fail loudly (gpu tests never skip silently)."""
    import torch

    if not torch.cuda.is_available():
        pytest.fail("gpu-marked test run without a visible HIP device")
    from irc_amd import _lib

    _lib.load()  # raises if libirc_hip.so is missing
    return torch.device("cuda:0")

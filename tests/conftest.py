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


def bf16_ulps(got, ref, floor):
    """Largest |got - ref| in bf16 ulps of the reference value: the ulp taken at
    max(|ref|, floor) (bf16 keeps 8 significant bits: ulp(x) = 2^(floor(log2 x) - 7)).
    The floor is the scale of the quantity (e.g. 1 for LayerNorm outputs): near zero a
    bf16 result carries the rounding of the O(floor) values it was computed from, not
    ulps of its own tiny magnitude.  Used for every bf16-output bound: an absolute bound
    on bf16 outputs is either loose at small values or fails at large ones."""
    got = np.asarray(got, dtype=np.float64)
    ref = np.asarray(ref, dtype=np.float64)
    ulp = np.exp2(np.floor(np.log2(np.maximum(np.abs(ref), floor))) - 7)
    return float(np.max(np.abs(got - ref) / ulp))


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

import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(REPO, "tests", "golden")
for p in (REPO, os.path.join(REPO, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)

import kcmc_amd  # noqa: E402,F401  (registers the package name)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels through the C ABI)")


def pytest_collection_modifyitems(config, items):
    try:
        import torch

        has_gpu = torch.cuda.is_available()
    except Exception:  # pragma: no cover
        has_gpu = False
    if has_gpu:
        return
    skip = pytest.mark.skip(reason="no GPU visible (run with -m gpu on the MI355X box)")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)


def distinct_frames(base, F):
    """F frames with pairwise different content: the base texture rolled by (37 f, 53 f)
    pixels, so that a tile that read another frame's staged data cannot match by accident."""
    return np.ascontiguousarray(np.stack([np.roll(base, (37 * f, 53 * f), axis=(0, 1)) for f in range(F)]))


def load_golden(name):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


@pytest.fixture(scope="session")
def golden():
    return load_golden


@pytest.fixture(scope="session")
def dev():
    import torch

    return torch.device("cuda", 0)

import os
import sys

import pytest

REPO = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
PKG = os.path.join(REPO, "graph-representation-learning_amd")
GOLDEN = os.path.join(REPO, "tests", "golden")
for p in (PKG, REPO, GOLDEN):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run on the GPU box via gpurun)")
    config.addinivalue_line("markers", "slow: longer-running CPU test")


def _has_gpu() -> bool:
    import torch

    return torch.cuda.is_available()


def pytest_collection_modifyitems(config, items):
    if any("gpu" in item.keywords for item in items) and not _has_gpu():
        skip = pytest.mark.skip(reason="no ROCm GPU visible")
        for item in items:
            if "gpu" in item.keywords:
                item.add_marker(skip)


@pytest.fixture(scope="session")
def golden():
    import numpy as np

    def load(name):
        return dict(np.load(os.path.join(GOLDEN, name), allow_pickle=False))

    return load


@pytest.fixture
def grl_option():
    """Set a libgrl path option (grl_set_option: the kernel-form hooks, e.g.
    grl_option("gemm_x6", 0)) for one test; every option it touched is
    restored afterwards."""
    from grl import _lib

    saved = {}

    def set_(name, value):
        if name not in saved:
            saved[name] = _lib.get_option(name)
        _lib.set_option(name, value)

    yield set_
    for name, value in saved.items():
        _lib.set_option(name, value)

import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: test needs an MI355X (HIP) device")
    config.addinivalue_line("markers", "slow: long-running test")


def pytest_collection_modifyitems(config, items):
    import torch
    if torch.cuda.is_available():
        return
    skip = pytest.mark.skip(reason="no GPU")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)


@pytest.fixture(autouse=True)
def _restore_gemm_modes():
    """A test that turns on deterministic mode (a trainer with deterministic = 1), forces a
    tile or switches the LDS-DMA kernels off must not leak that into the tests after it."""
    from cxxnet_amd.ops import gemm
    saved = (gemm._DET["on"], {k: set(v) if isinstance(v, set) else v for k, v in gemm._glds_cfg.items()})
    yield
    if gemm._DET["on"] != saved[0]:
        gemm.set_deterministic(saved[0])
    gemm._glds_cfg.clear()
    gemm._glds_cfg.update(saved[1])

import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "query-compiler-executor_amd")
for p in (PKG, os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box via gpurun)")
    config.addinivalue_line("markers", "slow: long-running (full-size) case")


@pytest.fixture(scope="session")
def ctx():
    """One libqe device context for the whole GPU session (native path only, no fallback)."""
    # torch's bundled HIP runtime must initialise before libqe's (tests use torch for device
    # buffers; the bench does the same)
    import torch
    torch.cuda.init()
    from qe import lib
    c = lib.Ctx(0)
    yield c
    c.close()

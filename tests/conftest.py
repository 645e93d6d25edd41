import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_DIR = os.path.join(REPO, "llama.cpp-quant-gemm_amd")
for p in (REPO, PKG_DIR, os.path.join(REPO, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU; parity tests through the C-ABI")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session")
def O():
    import oracle
    oracle.lib()
    return oracle


@pytest.fixture(scope="session")
def qg():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU test selected but no GPU is visible")
    import quant_gemm
    return quant_gemm

"""pytest setup: import paths and the `gpu` marker.

`-m "not gpu"` tests run on the CPU container (oracle vs golden vectors, host logic, C-ABI exports);
`-m gpu` tests are the parity tests proper and call the HIP kernels through libcp25.so.
"""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "cosmos-predict2.5_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels)")


@pytest.fixture(scope="session")
def device():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")

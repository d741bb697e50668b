import importlib
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_NAME = "radix-sort-merge-sort-cuda---lab-y-practicos-gpgpu-2023_amd"
for p in (REPO, os.path.join(REPO, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through liblabsort.so on cuda:0)")
    config.addinivalue_line("markers", "slow: full-size (2^28) cases")


@pytest.fixture(scope="session")
def oracle():
    import oracle as O  # test infrastructure (std::sort, generator, lab.cu restatement)
    O.build()
    return O


@pytest.fixture(scope="session")
def ls():
    """The product package (ctypes view of liblabsort.so)."""
    return importlib.import_module(PKG_NAME)


@pytest.fixture(scope="session")
def torch_gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU test selected but torch.cuda is not available")
    torch.cuda.set_device(0)
    return torch

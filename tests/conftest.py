import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libsheep_amd.so)")


@pytest.fixture(scope="session")
def oracle():
    from oracle import oracle as O

    O.lib()
    return O


@pytest.fixture(scope="session")
def hep_edges(oracle):
    return oracle.read_dat(os.path.join(GOLDEN, "hep-th.dat"))


@pytest.fixture(scope="session")
def gpu():
    """The product library on cuda:0; fails loudly (never skips) when the HIP build is missing."""
    import torch

    assert torch.cuda.is_available(), "GPU test needs a HIP device"
    from sheep_amd import capi

    capi.lib()
    capi.call("sheep_gpu_init", 0)
    return capi


@pytest.fixture
def options(gpu):
    """Set libsheep_amd tuning options (sheep_set_option) for one test; restored afterwards."""
    saved = {}

    def set_(**kw):
        for k, v in kw.items():
            old = gpu.set_option(k, v)
            saved.setdefault(k, old)

    yield set_
    for k, v in saved.items():
        gpu.set_option(k, v)

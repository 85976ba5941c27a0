import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "ntt-gpu-qtesla_amd"), os.path.join(ROOT, "oracle"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)

PARAM_SETS = ("ref", "p-I", "p-III")
# p-III's prime at n = 4096 / 8192: the multi-wave four-step kernels (ntt_large.hpp)
LARGE_SETS = ("p-III-4096", "p-III-8192")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP library)")
    config.addinivalue_line("markers", "slow: large-batch property checks")


@pytest.fixture(scope="session")
def oracle():
    import oracle as O
    if not os.path.exists(O.LIB_PATH):
        O.build()
    return O


@pytest.fixture(scope="session")
def ntt():
    import ntt_amd
    if not os.path.exists(ntt_amd.LIB_PATH):
        import __graft_entry__
        __graft_entry__.build()
    ntt_amd.lib()
    return ntt_amd


@pytest.fixture(scope="session")
def dev():
    import torch
    assert torch.cuda.is_available(), "gpu-marked tests need a GPU (the product has no CPU fallback)"
    return torch.device("cuda:0")

import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


@pytest.fixture(autouse=True)
def _release_hbm(request):
    """After every gpu test, hand the HBM it left in torch's caching
    allocator back to the device, so a later full-size test sees the whole
    card (a 128 GiB tensor held in the cache made the
    64 GiB every-ref test skip)."""
    yield
    if request.node.get_closest_marker("gpu") is None:
        return
    import gc
    import torch
    gc.collect()
    if torch.cuda.is_available():
        torch.cuda.synchronize()
        torch.cuda.empty_cache()


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI)")


@pytest.fixture(scope="session")
def O():
    """The CPU oracle (test infrastructure; oracle/oracle.h)."""
    from oracle import oracle
    oracle.build()
    return oracle


@pytest.fixture(scope="session")
def gpu():
    """The product path; skips nothing -- a gpu-marked test fails loudly if
    the library or the device is missing."""
    from glfs_amd import _native
    assert _native.device_count() > 0, "no HIP device visible"
    return _native

import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


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

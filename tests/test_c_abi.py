"""The C-ABI from plain C (tests/c/abi_test.c), compiled against
include/glfsx.h with gcc -Werror and linked to libglfsx.so: prototypes,
struct layout, status codes, the post callback, pageable buffers, panics,
strict error timing and cross-thread writer use, checked against the oracle
(test infrastructure).  The layout / no-fallback part runs without a GPU."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def abi_bin(O, tmp_path_factory):
    out = str(tmp_path_factory.mktemp("cabi") / "abi_test")
    libdir, odir = os.path.join(ROOT, "glfs_amd"), os.path.join(ROOT, "oracle")
    subprocess.check_call(
        ["gcc", "-std=c11", "-O1", "-Wall", "-Wextra", "-Werror", "-Wstrict-prototypes",
         "-I", os.path.join(ROOT, "include"), "-I", odir,
         os.path.join(ROOT, "tests", "c", "abi_test.c"),
         "-L", libdir, "-lglfsx", "-L", odir, "-loracle", "-lpthread",
         f"-Wl,-rpath,{libdir}", f"-Wl,-rpath,{odir}", "-o", out])
    return out


def test_c_consumer_layout_and_panics(abi_bin):
    p = subprocess.run([abi_bin, "layout"], capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stdout + p.stderr


@pytest.mark.gpu
def test_c_consumer_writer_vs_oracle(abi_bin):
    p = subprocess.run([abi_bin, "gpu"], capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stdout + p.stderr
    assert "abi_test gpu: ok" in p.stdout

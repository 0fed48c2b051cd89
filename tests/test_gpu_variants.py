"""Build variants that the shipped library no longer takes by default keep
producing the reference's bytes (the GLFSX_PIPE=0 fallback of the
CID pass must not rot).  __graft_entry__.build() builds them next to the
product (glfs_amd/libglfsx_<name>.so); each runs the headline's kernel shape
(2 GiB at 1 MiB blocks in one launch: 2048 workgroups, G = 4, no split) in a
child process, and its refs and ctext must equal the shipped library's and
the oracle's (digests of every byte)."""
import hashlib
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TOTAL, BS, SEED = 2 << 30, 1 << 20, 77
VARIANTS = ["pipe0"]


@pytest.fixture(scope="module")
def want(O):
    import ctypes
    n = TOTAL // BS
    data = O.fill_splitmix(TOTAL, SEED)
    refs = ctypes.create_string_buffer(64 * n)
    ct = ctypes.create_string_buffer(TOTAL)
    threads = min(16, os.cpu_count() or 1)
    O.lib().oracle_post_batch(refs, ct, bytes(range(32)), data, TOTAL, BS, None, threads)
    return {"refs": hashlib.sha256(refs.raw).hexdigest(),
            "ctext": hashlib.sha256(ct.raw).hexdigest()}


def _run(lib):
    env = dict(os.environ)
    if lib:
        env["GLFSX_LIB"] = lib
    out = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "variant_refs.py"),
                          str(TOTAL), str(BS), str(SEED)], env=env, capture_output=True,
                         text=True, timeout=240, check=True).stdout
    return json.loads(out.strip().splitlines()[-1])


def test_shipped_library_headline_shape(gpu, want):
    got = _run(None)
    assert (got["refs"], got["ctext"]) == (want["refs"], want["ctext"])


@pytest.mark.parametrize("name", VARIANTS)
def test_variant_build_parity(gpu, want, name):
    lib = os.path.join(ROOT, "glfs_amd", f"libglfsx_{name}.so")
    assert os.path.exists(lib), f"{lib} missing: __graft_entry__.build() builds it"
    got = _run(lib)
    assert got["lib"] == os.path.basename(lib)
    assert (got["refs"], got["ctext"]) == (want["refs"], want["ctext"])

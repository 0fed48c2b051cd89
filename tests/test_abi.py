"""The C-ABI library loads, exports exactly what include/glfsx.h declares, and
fails loudly (no CPU fallback) when no GPU is present.  CPU-only."""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "glfsx.h")


def header_symbols():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return set(re.findall(r"\b(glfsx_[a-z0-9_]+)\s*\(", txt)) - {"glfsx_post_fn"}


def test_header_matches_binding_and_exports():
    from glfs_amd import _native
    syms = header_symbols()
    assert syms == set(_native.SIGNATURES), syms ^ set(_native.SIGNATURES)
    out = subprocess.check_output(["nm", "-D", "--defined-only", _native.LIB_PATH],
                                  text=True)
    exported = set(re.findall(r"\bT (glfsx_[a-z0-9_]+)", out))
    assert syms <= exported, syms - exported


def test_library_is_gfx950():
    from glfs_amd import _native
    out = subprocess.check_output(
        ["/opt/rocm/lib/llvm/bin/clang-offload-bundler", "--list", "--type=o",
         f"--input={_native.LIB_PATH}"], text=True, stderr=subprocess.STDOUT) \
        if os.path.exists("/opt/rocm/lib/llvm/bin/clang-offload-bundler") else ""
    data = open(_native.LIB_PATH, "rb").read()
    assert b"gfx950" in data or "gfx950" in out


def test_depth_matches_oracle(O):
    """blob.go:256-264 is host-side integer shape math."""
    from glfs_amd import bigblob
    for bs in (128, 1000, 1024, 1 << 20, 2 << 20):
        bf = bs // 64
        for size in (0, 1, bs, bs + 1, bf * bs, bf * bs + 1, bf * bf * bs + 1, 10 ** 12):
            assert bigblob.depth(size, bs) == O.depth(size, bs)
        assert bigblob.branching_factor(bs) == bf


def test_ref_marshal_roundtrip():
    """bigblob/ref_test.go:27-40 TestRefMarshal (host-side layout)."""
    from glfs_amd.bigblob import Ref
    r = Ref(bytes(range(32)), bytes(range(32, 64)))
    assert Ref.from_bytes(r.marshal_binary()) == r
    with pytest.raises(ValueError):
        Ref.from_bytes(b"x" * 63)


def test_no_cpu_fallback_without_gpu():
    from glfs_amd import _native, bigblob
    if _native.device_count() > 0:
        pytest.skip("GPU present")
    with pytest.raises(_native.DeviceError):
        bigblob.derive_key(bytes(32), b"raw")
    with pytest.raises(_native.DeviceError):
        bigblob.Machine(1024).create(bigblob.MemStore(1024), None, b"abc")


def test_library_reads_only_the_documented_knobs():
    """the library reads five GLFSX_* variables, all
    tuning (tests/test_gpu_knobs.py runs each at a non-default value); every
    getenv in its sources names one of them."""
    knobs = {"GLFSX_BATCH_MIB", "GLFSX_SLOTS", "GLFSX_SPIN_US", "GLFSX_NUMA",
             "GLFSX_READ_THREADS"}
    csrc = os.path.join(ROOT, "glfs_amd", "csrc")
    names, calls = set(), 0
    for f in os.listdir(csrc):
        if f.endswith((".cpp", ".hip", ".h")):
            src = open(os.path.join(csrc, f)).read()
            names |= set(re.findall(r'getenv\("(GLFSX_\w+)"\)', src))
            calls += src.count("getenv(")
    assert names == knobs, names ^ knobs
    assert calls == len(knobs)


def test_file_route_only_for_plain_files(tmp_path):
    """Writer.read_from takes the parallel pread route only for a plain file
    (io.FileIO, or a buffered reader over one): a gzip / bz2 / lzma file
    reports the compressed file's descriptor but a decompressed position, so
    it must go through readinto."""
    import bz2
    import gzip
    import io
    import lzma
    from glfs_amd.bigblob import _regular_fd
    p = tmp_path / "f.bin"
    p.write_bytes(b"x" * 1000)
    with open(p, "rb") as f:
        assert _regular_fd(f) == f.fileno()
    with open(p, "rb", buffering=0) as f:
        assert _regular_fd(f) == f.fileno()
    with open(p, "r+b") as f:
        assert _regular_fd(f) == f.fileno()
    for opener, name in ((gzip.open, "f.gz"), (bz2.open, "f.bz2"), (lzma.open, "f.xz")):
        q = tmp_path / name
        with opener(q, "wb") as f:
            f.write(b"y" * 5000)
        with opener(q, "rb") as f:
            assert _regular_fd(f) is None, name
    assert _regular_fd(io.BytesIO(b"abc")) is None
    r, w = os.pipe()
    try:
        with os.fdopen(r, "rb", closefd=False) as f:
            assert _regular_fd(f) is None
    finally:
        os.close(r)
        os.close(w)


def test_writer_panics_mirror_reference():
    """blob.go:90-95 panics surface as Panic, before any device work."""
    from glfs_amd import _native, bigblob
    with pytest.raises(_native.Panic, match="2097152 > maxSize 1048576"):
        bigblob.Machine(2 << 20).new_writer(bigblob.MemStore(1 << 20))
    with pytest.raises(_native.Panic, match="< 128"):
        bigblob.Machine(100).new_writer(bigblob.MemStore(1 << 20))
    with pytest.raises(_native.Panic):
        bigblob.Machine(-1)


def test_postbench_harness_rejects_bad_arguments():
    """tools/libpostbench.so (bench.py's postblob_concurrency leg): built by
    build(), loads without a GPU, and refuses a run with no entry points or
    no threads before starting any (no GPU call)."""
    import ctypes
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    path = os.path.join(root, "tools", "libpostbench.so")
    if not os.path.exists(path):
        pytest.skip("tools/libpostbench.so not built")
    lib = ctypes.CDLL(path)
    lib.postbench_run.restype = ctypes.c_int
    lib.postbench_run.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_int, ctypes.c_uint64,
                                                           ctypes.c_int, ctypes.c_char_p,
                                                           ctypes.c_int, ctypes.c_void_p]
    out = (ctypes.c_double * 5)()
    assert lib.postbench_run(None, None, None, 4, 4096, 10, bytes(32), 0, out) == -1
    assert lib.postbench_run(1, 1, 1, 0, 4096, 10, bytes(32), 0, out) == -1
    assert lib.postbench_run(1, 1, 1, 4, 4096, 0, bytes(32), 0, out) == -1

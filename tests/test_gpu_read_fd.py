"""bigblob.Create fed by a file or an io.ReaderAt (bigblob/blob.go:209-217;
glfs.go:53 io.Copy): glfsx_writer_read_fd / glfsx_writer_read_at read each
batch straight into the Writer's pinned staging with several threads while
earlier batches hash.  The Post log (kind, ref, ctext) and the root must be
the oracle writer's over the same bytes, for one lane and for three lanes of
the one GPU; offsets, short files, read errors and the Python API's file
route are covered too.
"""
import ctypes
import hashlib
import os
import tempfile

import pytest

from test_gpu_multi import _oracle_post_log

pytestmark = pytest.mark.gpu

MIB = 1 << 20


def _sink_log(N):
    log = []

    @N.POST_FN
    def sink(_ctx, kind, ref, ct, n):
        log.append((kind, ctypes.string_at(ref, 64), n,
                    hashlib.sha256(ctypes.string_at(ct, n)).digest()))
        return 0
    return sink, log


def _writer(N, bs, sink, devs=None):
    err = ctypes.c_int(0)
    w = N.lib.glfsx_writer_new(bs, bs, None, None, sink, None, ctypes.byref(err))
    assert w, N.last_error()
    if devs:
        N.check(N.lib.glfsx_writer_set_devices(w, (ctypes.c_int * len(devs))(*devs), len(devs)))
    return w


def _finish(N, w):
    root = N.glfsx_root()
    rc = N.lib.glfsx_writer_finish(w, ctypes.byref(root))
    N.check(rc, (N.lib.glfsx_writer_error(w) or b"").decode())
    return bytes(root.ref)


@pytest.fixture(scope="module")
def file300(O):
    data = O.fill_splitmix(300 * MIB + 12345, 31)
    fd, path = tempfile.mkstemp(prefix="glfsx_rfd_")
    with os.fdopen(fd, "wb") as f:
        f.write(data)
    yield path, data
    os.unlink(path)


@pytest.mark.parametrize("devs", [None, [0, 0, 0]])
def test_read_fd_post_log_vs_oracle(gpu, O, file300, devs):
    """300 MiB + 12345 B at 1 MiB blocks from a file: 301 data Posts + 1
    index Post equal to the oracle writer's."""
    N = gpu
    path, data = file300
    want_root, want_log = _oracle_post_log(O, data, MIB)
    sink, log = _sink_log(N)
    w = _writer(N, MIB, sink, devs)
    fd = os.open(path, os.O_RDONLY)
    try:
        got = ctypes.c_uint64()
        rc = N.lib.glfsx_writer_read_fd(w, fd, 0, (1 << 64) - 1, ctypes.byref(got))
        N.check(rc, (N.lib.glfsx_writer_error(w) or b"").decode())
        assert got.value == len(data)
        assert _finish(N, w) == want_root
    finally:
        os.close(fd)
        N.lib.glfsx_writer_free(w)
    assert log == want_log


def test_read_fd_offset_and_mixed_writes(gpu, O, file300):
    """A Write, then bytes [1000, 1000 + 77 MiB + 5) of the file, then another
    Write: the blob is the concatenation (blocks straddle the pieces)."""
    N = gpu
    path, data = file300
    head, tail = b"h" * 333, b"t" * (3 * MIB + 1)
    n = 77 * MIB + 5
    blob = head + data[1000:1000 + n] + tail
    want_root, want_log = _oracle_post_log(O, blob, 64 << 10)
    sink, log = _sink_log(N)
    w = _writer(N, 64 << 10, sink)
    fd = os.open(path, os.O_RDONLY)
    try:
        N.check(N.lib.glfsx_writer_write(w, head, len(head)))
        got = ctypes.c_uint64()
        N.check(N.lib.glfsx_writer_read_fd(w, fd, 1000, n, ctypes.byref(got)))
        assert got.value == n
        N.check(N.lib.glfsx_writer_write(w, tail, len(tail)))
        assert _finish(N, w) == want_root
    finally:
        os.close(fd)
        N.lib.glfsx_writer_free(w)
    assert log == want_log


def test_read_fd_short_file_and_errors(gpu, O, file300):
    """n past the end takes what is there; a bad descriptor is GLFSX_E_ARG;
    a failing ReaderAt is GLFSX_E_IO with the bytes before it taken and the
    writer still usable."""
    N = gpu
    path, data = file300
    sink, log = _sink_log(N)
    w = _writer(N, MIB, sink)
    fd = os.open(path, os.O_RDONLY)
    try:
        got = ctypes.c_uint64()
        start = len(data) - 5 * MIB - 7
        N.check(N.lib.glfsx_writer_read_fd(w, fd, start, 64 * MIB, ctypes.byref(got)))
        assert got.value == 5 * MIB + 7
        assert N.lib.glfsx_writer_read_fd(w, -1, 0, 10, ctypes.byref(got)) == N.GLFSX_E_ARG
        calls = []

        def bad(_ctx, buf, ln, off):
            calls.append(off)
            return -5
        cb = N.READ_AT_FN(bad)
        assert N.lib.glfsx_writer_read_at(w, cb, None, 0, 10 * MIB, ctypes.byref(got)) == \
            N.GLFSX_E_IO
        assert got.value == 0 and calls
        assert _finish(N, w) == _oracle_post_log(O, data[start:], MIB)[0]
    finally:
        os.close(fd)
        N.lib.glfsx_writer_free(w)


def test_read_at_callback_and_python_file_route(gpu, O, file300):
    """An io.ReaderAt as a callback (called from several threads), and
    bigblob.Machine.create over an open file (the Python io.Copy takes the
    file route and leaves the file positioned after what it read)."""
    from glfs_amd import bigblob
    N = gpu
    path, data = file300
    n = 130 * MIB + 3
    want_root, want_log = _oracle_post_log(O, data[:n], MIB)
    st = bigblob.MemStore(MIB)
    m = bigblob.Machine(MIB)
    w = m.new_writer(st)
    mv = memoryview(data)

    def read_at(buf, off):
        k = max(0, min(len(buf), n - off))
        buf[:k] = mv[off:off + k]
        return k
    assert w.read_at(read_at) == n
    root = w.finish()
    w.close()
    assert root.ref.marshal_binary() == want_root
    with open(path, "rb") as f:
        f.seek(7)
        f.read(10)                    # buffered read: the logical position is 17
        st2 = bigblob.MemStore(MIB)
        r2 = m.create(st2, None, f)
        assert f.tell() == len(data)
    assert r2.ref.marshal_binary() == _oracle_post_log(O, data[17:], MIB)[0]
    assert r2.size == len(data) - 17


def test_create_from_gzip_file(gpu, O, tmp_path):
    """bigblob.Machine.create over gzip.open(path): the blob is the
    DECOMPRESSED bytes (the reader's readinto), never the compressed file's
    bytes at the decompressed offset."""
    import gzip
    from glfs_amd import bigblob
    data = O.fill_splitmix(5 * MIB + 77, 8)
    p = tmp_path / "blob.gz"
    with gzip.open(p, "wb", compresslevel=1) as f:
        f.write(data)
    m = bigblob.Machine(MIB)
    with gzip.open(p, "rb") as f:
        f.read(5)                                  # a decompressed position of 5
        r = m.create(bigblob.MemStore(MIB), None, f)
    assert r.ref.marshal_binary() == _oracle_post_log(O, data[5:], MIB)[0]
    assert r.size == len(data) - 5


def test_read_at_short_reads_and_strict(gpu, O, file300):
    """A ReaderAt that returns at most 100,003 bytes per call (short reads at
    every piece boundary, as a network-backed io.ReaderAt may) into a strict
    writer over two lanes of the one GPU: the Post log equals the oracle's."""
    N = gpu
    path, data = file300
    n = 97 * MIB + 11
    want_root, want_log = _oracle_post_log(O, data[:n], MIB)
    sink, log = _sink_log(N)
    w = _writer(N, MIB, sink, [0, 0])
    N.check(N.lib.glfsx_writer_set_strict(w, 1))
    mv = memoryview(data)

    def short(_ctx, buf, ln, off):
        k = max(0, min(ln, 100_003, n - off))
        ctypes.memmove(buf, bytes(mv[off:off + k]), k)
        return k
    cb = N.READ_AT_FN(short)
    try:
        got = ctypes.c_uint64()
        rc = N.lib.glfsx_writer_read_at(w, cb, None, 0, (1 << 64) - 1, ctypes.byref(got))
        N.check(rc, (N.lib.glfsx_writer_error(w) or b"").decode())
        assert got.value == n
        assert _finish(N, w) == want_root
    finally:
        N.lib.glfsx_writer_free(w)
    assert log == want_log

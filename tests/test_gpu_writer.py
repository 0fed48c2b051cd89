"""bigblob Writer semantics through the C-ABI (blob.go:71-206): strict error
timing (the Write that fills a failing block returns the store error, and no
Post follows the failing one), flush, and a writer driven from several host
threads in turn (a goroutine migrating between OS threads: ADVICE r1)."""
import ctypes
import random
import threading

import pytest

pytestmark = pytest.mark.gpu


def _oracle_fail_run(O, data, bs, pieces, fail_at):
    """The reference Writer (oracle restatement) over `pieces`, with a store
    whose fail_at-th Post (1-based) fails.  Returns (index of the Write that
    returned the error or None, 'finish' if Finish did, posts delivered)."""
    L = O.lib()
    posts = []

    def sink(_ctx, kind, ref, ct, n):
        posts.append((kind, ctypes.string_at(ref, 64)))
        return 1 if len(posts) == fail_at else 0

    cb = O.SINK_FN(sink)
    err = ctypes.c_int(0)
    w = L.oracle_writer_new(bs, bs, None, None, cb, None, ctypes.byref(err))
    try:
        off = 0
        for i, p in enumerate(pieces):
            piece = data[off:off + p]
            off += p
            if L.oracle_writer_write(w, piece, len(piece)) != 0:
                return i, posts
        root = ctypes.create_string_buffer(64)
        size, bsz = ctypes.c_uint64(), ctypes.c_uint64()
        if L.oracle_writer_finish(w, root, ctypes.byref(size), ctypes.byref(bsz)) != 0:
            return "finish", posts
        return None, posts
    finally:
        L.oracle_writer_free(w)


class _FailingStore:
    def __init__(self, bs, fail_at):
        from glfs_amd import bigblob
        self.inner = bigblob.MemStore(bs)
        self.fail_at = fail_at
        self.n = 0

    def max_size(self):
        return self.inner.max_size()

    def post(self, ct, ref, kind=0):
        self.n += 1
        self.inner.post(ct, ref, kind)
        if self.n == self.fail_at:
            raise IOError(f"post {self.n} refused")


@pytest.mark.parametrize("fail_at", [1, 3, 16, 17, 18, 35, 37, 41])
def test_strict_error_timing_matches_reference(gpu, O, fail_at):
    """blob.go:120-133 + 152-182: with strict timing the GPU writer returns
    the store error from the same Write (or Finish) as the reference, after
    exactly the same Posts, in the same order."""
    from glfs_amd import bigblob
    bs = 1024                       # bf = 16: index posts interleave
    data = O.fill_splitmix(40 * bs + 300, 19)
    pieces = [3000, 1, 5000, 17 * bs, 2, 9000]
    pieces.append(len(data) - sum(pieces))
    want_at, want_posts = _oracle_fail_run(O, data, bs, pieces, fail_at)
    st = _FailingStore(bs, fail_at)
    w = bigblob.Machine(bs).new_writer(st, None, strict=True)
    got_at = None
    try:
        off = 0
        for i, p in enumerate(pieces):
            try:
                w.write(data[off:off + p])
            except bigblob.StoreError:
                got_at = i
                break
            off += p
        else:
            try:
                w.finish()
            except bigblob.StoreError:
                got_at = "finish"
    finally:
        w.close()
    assert got_at == want_at
    assert [(k, r) for k, r, _ in st.inner.log] == want_posts


def test_default_error_no_posts_after_failure(gpu, O):
    """Default (pipelined) timing: the error may surface at a later Write,
    but the Posts delivered are still exactly the reference's prefix."""
    from glfs_amd import bigblob
    bs = 4096
    data = O.fill_splitmix(300 * bs + 5, 23)
    _, want_posts = _oracle_fail_run(O, data, bs, [len(data)], 130)
    st = _FailingStore(bs, 130)
    w = bigblob.Machine(bs).new_writer(st, None)
    with pytest.raises(bigblob.StoreError):
        w.write(data)
        w.finish()
    w.close()
    assert [(k, r) for k, r, _ in st.inner.log] == want_posts


@pytest.mark.parametrize("fail_at", [1, 17, 35, 41, 43])
def test_strict_read_from_returns_the_io_copy_error(gpu, O, fail_at):
    """The Go binding's default (GLFSX_STRICT=1) ReadFrom: pipelined inside
    the call, its Posts flushed before it returns.  The reference's io.Copy
    (32 KiB Writes, blob.go:120-133) returns a store error from the copy when
    the failing Post belongs to a block the input completed, else Finish
    does; the GPU writer's read_from / finish must fail at the same place,
    after exactly the same Posts."""
    import io
    from glfs_amd import bigblob
    bs = 1024                       # bf = 16: index posts interleave
    data = O.fill_splitmix(40 * bs + 300, 29)
    pieces = [32768] * (len(data) // 32768) + [len(data) % 32768]
    want_at, want_posts = _oracle_fail_run(O, data, bs, pieces, fail_at)
    want = None if want_at is None else ("finish" if want_at == "finish" else "copy")
    st = _FailingStore(bs, fail_at)
    w = bigblob.Machine(bs).new_writer(st, None, strict=True)
    got = None
    try:
        try:
            assert w.read_from(io.BytesIO(data)) == len(data)
        except bigblob.StoreError:
            got = "copy"
        if got is None:
            try:
                w.finish()
            except bigblob.StoreError:
                got = "finish"
    finally:
        w.close()
    assert got == want
    assert [(k, r) for k, r, _ in st.inner.log] == want_posts


def test_flush_delivers_complete_blocks(gpu, O):
    from glfs_amd import bigblob
    bs = 1 << 20
    data = O.fill_splitmix(5 * bs + 10, 3)
    _, _, _, want = O.create(data, bs)
    st = bigblob.MemStore(bs)
    w = bigblob.Machine(bs).new_writer(st, None)
    w.write(data[:3 * bs + 7])
    w.flush()
    assert [r for _, r, _ in st.log] == [r for _, r, _, _ in want[:3]]
    w.write(data[3 * bs + 7:])
    root = w.finish()
    w.close()
    assert [r for _, r, _ in st.log] == [r for _, r, _, _ in want]
    assert root.ref.marshal_binary() == O.create(data, bs)[0]


def test_writer_across_threads(gpu, O):
    """One writer created, written and finished on three different threads
    while other threads run their own writers and one-shot posts; every
    root and Post sequence equals the reference's (the writer no
    longer borrows the creating thread's stream and staging)."""
    from glfs_amd import _native as N, bigblob
    bs = 64 << 10
    jobs = [O.fill_splitmix(n, 100 + i) for i, n in
            enumerate([40 * bs + 11, 17 * bs, 3 * bs + 1, 70 * bs + 999])]
    results = {}
    errors = []

    def run_in_thread(fn):
        t = threading.Thread(target=fn)
        t.start()
        t.join()

    def migrating(i):
        data = jobs[i]
        st = bigblob.MemStore(bs)
        box = {}
        run_in_thread(lambda: box.setdefault("w", bigblob.Machine(bs).new_writer(st, None)))
        rng = random.Random(i)
        off = 0
        while off < len(data):
            p = rng.randrange(1, 6 * bs)
            run_in_thread(lambda o=off, p=p: box["w"].write(data[o:o + p]))
            off += p
        run_in_thread(lambda: box.setdefault("root", box["w"].finish()))
        run_in_thread(lambda: box["w"].close())
        results[i] = (box["root"], st)

    def noise():
        try:
            for k in range(20):
                m = O.fill_splitmix(5000 + k, k)
                ref = bigblob.Machine(1024).post(bigblob.MemStore(1 << 20), bytes(32), m)
                assert ref.marshal_binary() == O.post(bytes(32), m)[0]
        except Exception as e:  # surfaced below
            errors.append(e)

    ths = [threading.Thread(target=migrating, args=(i,)) for i in range(len(jobs))]
    ths += [threading.Thread(target=noise) for _ in range(2)]
    [t.start() for t in ths]
    [t.join() for t in ths]
    assert not errors, errors
    for i, data in enumerate(jobs):
        root, st = results[i]
        want_root, _, _, want_posts = O.create(data, bs)
        assert root.ref.marshal_binary() == want_root, i
        assert [r for _, r, _ in st.log] == [r for _, r, _, _ in want_posts], i
    assert N.device_count() > 0


def test_write_device_mixed_with_host_writes(gpu, O):
    """glfsx_writer_write_device: bytes from HBM in random pieces, mixed
    with host writes (the staging moves between host and device), across
    batch boundaries and index posts; root and Post log == the reference
    writer's.  The producer stream reuses its buffer right after each call:
    the writer must have consumed the bytes by then (stream ordering)."""
    import torch
    from glfs_amd import _native as N, bigblob
    bs = 64 << 10
    size = 1100 * bs + 12345           # > one 64 MiB batch, 1 index node + tail
    data = O.fill_splitmix(size, 31)
    want_root, _, _, want_posts = O.create(data, bs)
    st = bigblob.MemStore(bs)
    w = bigblob.Machine(bs).new_writer(st, None)
    s = torch.cuda.Stream()
    buf = torch.empty(8 << 20, dtype=torch.uint8, device="cuda")
    rng = random.Random(5)
    off = 0
    while off < size:
        p = min(rng.randrange(1, 6 << 20), size - off)
        piece = data[off:off + p]
        if rng.random() < 0.3:
            w.write(piece)
        else:
            with torch.cuda.stream(s):
                buf[:p].copy_(torch.frombuffer(bytearray(piece), dtype=torch.uint8),
                              non_blocking=False)
                w.write_device(buf.data_ptr(), p, ctypes.c_void_p(s.cuda_stream))
                buf.fill_(0xEE)            # reuse at once, ordered after the write
        off += p
    root = w.finish()
    w.close()
    assert root.ref.marshal_binary() == want_root
    assert [(k, r) for k, r, _ in st.log] == [(k, r) for k, r, _, _ in want_posts]


def test_concat_write_ctext_vs_oracle(gpu, O):
    """blob.go:333-345 Concat at 1 MiB blocks over roots of ragged sizes
    (single-block, multi-block with an index node, empty): the data blocks
    go to the new Writer as ciphertext and are decrypted on the GPU into its
    staging; root == the oracle's Create of the joined bytes."""
    from glfs_amd import bigblob
    bs = 1 << 20
    m = bigblob.Machine(bs)
    st = bigblob.NativeStore(bs, "trust")
    parts = [O.fill_splitmix(n, 70 + i) for i, n in
             enumerate([3 * bs + 777, 0, 100, bs, 70 * bs + 5])]
    roots = [m.create(st, None, p) for p in parts]
    got = m.concat(st, 4096, None, *roots)
    want = O.create(b"".join(parts), bs)[0]
    assert got.ref.marshal_binary() == want
    assert got.size == sum(map(len, parts))
    assert bigblob.read_all(st, got) == b"".join(parts)


def test_concat_from_store_memory_many_slabs(gpu, O):
    """Concat from a NativeStore takes each ciphertext block straight from
    the store's memory (glfsx_writer_write_ctext_blocks: 64 MiB slabs of
    scattered blocks gathered into two pinned buffers in turn): 200 MiB
    (four slabs, so both buffers are reused) plus a ragged second root ==
    the oracle's Create of the joined bytes, and == the contiguous route
    (a MemStore: gathered in Python, glfsx_writer_write_ctext)."""
    from glfs_amd import bigblob
    bs = 1 << 20
    m = bigblob.Machine(bs)
    parts = [O.fill_splitmix(200 * bs + 12345, 91), O.fill_splitmix(3 * bs + 7, 92)]
    st = bigblob.NativeStore(bs, "trust")
    roots = [m.create(st, None, p) for p in parts]
    got = m.concat(st, bs, None, *roots)
    want = O.create(b"".join(parts), bs)[0]
    assert got.ref.marshal_binary() == want
    ms = bigblob.MemStore(bs)
    roots2 = [m.create(ms, None, p) for p in parts]
    assert m.concat(ms, bs, None, *roots2).ref.marshal_binary() == want


class _ChunkyReader:
    """An io.Reader whose Reads return random amounts (1 B .. 3 MiB), read
    into the caller's buffer (readinto), like a pipe or socket."""

    def __init__(self, data, seed):
        self.data, self.off = memoryview(data), 0
        self.rng = random.Random(seed)

    def readinto(self, buf):
        n = min(len(buf), len(self.data) - self.off, self.rng.choice([1, 4096, 65536, 1 << 20,
                                                                     3 << 20, 777_777]))
        buf[:n] = self.data[self.off:self.off + n]
        self.off += n
        return n


@pytest.mark.parametrize("strict", [False, True])
def test_read_from_vs_oracle(gpu, O, strict):
    """Writer.ReadFrom (glfsx_writer_reserve / _commit: the reader fills the
    pinned staging, io.Copy's fast path in Create): the Post log (kind,
    ref, ctext) and root equal the oracle writer's, with Reads of random
    sizes, pipelined and strict."""
    from glfs_amd import bigblob
    bs = 1 << 20
    data = O.fill_splitmix(70 * bs + 4321, 31)
    want_root, _, _, want = O.create(data, bs)
    st = bigblob.MemStore(bs)
    w = bigblob.Machine(bs).new_writer(st, None, strict=strict)
    try:
        assert w.read_from(_ChunkyReader(data, 5)) == len(data)
        root = w.finish()
    finally:
        w.close()
    assert root.ref.marshal_binary() == want_root and root.size == len(data)
    assert [(k, r) for k, r, _ in st.log] == [(k, r) for k, r, _, _ in want]
    for (k, r, n), (_, _, _, ct) in zip(st.log, want):
        assert st.blobs[r[:32]] == ct


def test_read_from_store_error(gpu, O):
    """A store error during ReadFrom: raised, and the Posts delivered are the
    reference's prefix (no Post after the failing one)."""
    from glfs_amd import bigblob
    bs = 4096
    data = O.fill_splitmix(200 * bs + 5, 37)
    _, want_posts = _oracle_fail_run(O, data, bs, [len(data)], 90)
    st = _FailingStore(bs, 90)
    w = bigblob.Machine(bs).new_writer(st, None, strict=True)
    with pytest.raises(bigblob.StoreError):
        w.read_from(_ChunkyReader(data, 7))
        w.finish()
    w.close()
    assert [(k, r) for k, r, _ in st.inner.log] == want_posts


def test_commit_more_than_reserved_fails(gpu):
    N = gpu
    err = ctypes.c_int()
    w = N.lib.glfsx_writer_new(1 << 20, 1 << 20, None, None, N.POST_FN(0), None,
                               ctypes.byref(err))
    try:
        buf, cap = ctypes.c_void_p(), ctypes.c_uint64()
        assert N.lib.glfsx_writer_reserve(w, ctypes.byref(buf), ctypes.byref(cap)) == 0
        assert cap.value == 64 << 20 and buf.value
        assert N.lib.glfsx_writer_commit(w, cap.value + 1) == N.GLFSX_E_ARG
    finally:
        N.lib.glfsx_writer_free(w)

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

"""One-shot posts (launch_one / k_one): a message of at most 64 KiB posted in
one launch straight from pinned staging; up to 4 MiB in two launches over
64 KiB spans (launch_med: k_med_dek / k_med_cid, last-arriving workgroup
merges); concurrent callers coalesced into shared launches (glfsx.cpp
one_post).  Every ref and ctext == the oracle's
ref.go:98 post(); Writers whose tail blocks and index nodes take this route
(block sizes <= 4 MiB) == the oracle Writer (blob.go:85-206), Post order
included."""
import ctypes
import os
import random
import threading

import pytest

pytestmark = pytest.mark.gpu

EDGES = [0, 1, 15, 16, 17, 63, 64, 65, 1023, 1024, 1025, 2047, 4096, 4097,
         16383, 16384, 16385, 32768 + 7, 65535, 65536]
MEDIUM = [65537, 65536 + 1024, 131072, 131073, 200000, (1 << 20) - 1, 1 << 20,
          (2 << 20) + 5, (4 << 20) - 64, 4 << 20]


def _gpu_post(N, salt, data, cid_key=None):
    ct = ctypes.create_string_buffer(max(len(data), 1))
    ref = ctypes.create_string_buffer(64)
    N.check(N.lib.glfsx_post(salt, data, len(data), ct, ref, cid_key))
    return ref.raw, ct.raw[:len(data)]


@pytest.mark.parametrize("keyed", [False, True])
def test_one_shot_post_edges(gpu, O, keyed):
    rng = random.Random(11 + keyed)
    for n in EDGES:
        salt = rng.randbytes(32)
        key = rng.randbytes(32) if keyed else None
        data = rng.randbytes(n)
        assert _gpu_post(gpu, salt, data, key) == O.post(salt, data, key), n


@pytest.mark.parametrize("keyed", [False, True])
def test_medium_post_edges(gpu, O, keyed):
    """64 KiB < n <= 4 MiB: the two-launch route (spans of 64 KiB, the last
    one partial; chunk counters continue across spans)."""
    rng = random.Random(21 + keyed)
    for n in MEDIUM:
        salt = rng.randbytes(32)
        key = rng.randbytes(32) if keyed else None
        data = rng.randbytes(n)
        assert _gpu_post(gpu, salt, data, key) == O.post(salt, data, key), n


def test_one_shot_post_unaligned_source(gpu, O):
    """The caller's bytes at odd addresses (copied into aligned staging)."""
    rng = random.Random(3)
    buf = rng.randbytes(70000)
    salt = rng.randbytes(32)
    for off, n in [(1, 100), (3, 4096), (7, 65536), (13, 0)]:
        view = (ctypes.c_char * n).from_buffer_copy(buf[off:off + n]) if n else b""
        data = bytes(view)
        assert _gpu_post(gpu, salt, data) == O.post(salt, data), (off, n)


@pytest.mark.parametrize("keyed", [False, True])
@pytest.mark.parametrize("bs", [1024, 4096, 65536, 1 << 20, 4 << 20])
def test_writer_small_blocks_one_shot(gpu, O, bs, keyed):
    """Tail blocks and every index node (bs <= 4 MiB) go through one-shot
    posts (index nodes from their refs alone, the rest read as zero): roots
    and the full Post log (kind, ref, ctext) == the oracle."""
    from glfs_amd import bigblob
    rng = random.Random(bs)
    sizes = [0, 1, bs - 1, bs, bs + 1, 3 * bs + 5]
    if bs <= 65536:
        sizes.append((bs // 64 + 2) * bs + 17)  # a full index node, then a second level
    for size in sizes:
        data = rng.randbytes(size)
        salt = rng.randbytes(32)
        key = rng.randbytes(32) if keyed else None     # keyed store CID
        want_root, _, _, want_posts = O.create(data, bs, salt=salt, cid_key=key)
        st = bigblob.MemStore(bs)
        w = bigblob.Machine(bs).new_writer(st, salt, key)
        w.write(data)
        root = w.finish()
        w.close()
        assert root.ref.marshal_binary() == want_root, (bs, size)
        assert [(k, r, n) for k, r, n in st.log] == \
               [(k, r, n) for k, r, n, _ in want_posts], (bs, size)
        for _, r, _, c in want_posts:
            assert st.blobs[r[:32]] == c, (bs, size)


def test_concurrent_one_shot_posts(gpu, O):
    """16 threads posting ragged small messages at once (coalesced launches
    of many workgroups): every result == the oracle."""
    errors = []

    def worker(t):
        try:
            from glfs_amd import _native as N
            N.check(N.lib.glfsx_set_device(0))
            rng = random.Random(1000 + t)
            for _ in range(60):
                n = rng.choice([0, 5, 64, 1000, 4096, 9000, 20000, 65536, 70000,
                                (1 << 20) + 3])
                salt = rng.randbytes(32)
                key = rng.randbytes(32) if rng.random() < 0.3 else None
                data = rng.randbytes(n)
                got = _gpu_post(N, salt, data, key)
                if got != O.post(salt, data, key):
                    errors.append((t, n))
        except Exception as e:  # surfaced below
            errors.append(e)

    th = [threading.Thread(target=worker, args=(t,)) for t in range(16)]
    [t.start() for t in th]
    [t.join() for t in th]
    assert not errors, errors[:5]


def test_many_waiters_one_stats(gpu, O):
    """64 threads posting small messages at once: more callers than the
    poster lets spin (the rest sleep between polls), so sleepers, spinners
    and leaders mix; every result == the oracle, and glfsx_one_stats counts
    every request once (launches <= requests)."""
    from glfs_amd import _native as N
    N.check(N.lib.glfsx_one_stats(1, None))
    errors = []
    per, threads = 25, 64

    def worker(t):
        try:
            N.check(N.lib.glfsx_set_device(0))
            rng = random.Random(5000 + t)
            for _ in range(per):
                n = rng.choice([0, 9, 100, 4096, 5000, 16384])
                salt = rng.randbytes(32)
                data = rng.randbytes(n)
                if _gpu_post(N, salt, data) != O.post(salt, data):
                    errors.append((t, n))
        except Exception as e:
            errors.append(e)

    th = [threading.Thread(target=worker, args=(t,)) for t in range(threads)]
    [t.start() for t in th]
    [t.join() for t in th]
    assert not errors, errors[:5]
    st = (ctypes.c_uint64 * 3)()
    N.check(N.lib.glfsx_one_stats(0, st))
    assert st[1] == per * threads
    assert 1 <= st[0] <= st[1]


def test_concurrent_small_creates(gpu, O):
    """glfs.PostBlob-shaped calls (glfsx_create, one Writer per blob) from 12
    threads, with the blob type salt: roots == the oracle's Create."""
    from glfs_amd import _native as N, glfs
    salt = glfs.Machine().make_salt("blob")
    bs = 2 << 20
    errors = []

    def worker(t):
        try:
            N.check(N.lib.glfsx_set_device(0))
            rng = random.Random(77 + t)
            counts, root = (ctypes.c_uint64 * 2)(), N.glfsx_root()
            sink = ctypes.cast(N.lib.glfsx_sink_count, N.POST_FN)
            for _ in range(40):
                data = rng.randbytes(rng.choice([0, 9, 4096, 70000, (1 << 20) + 1,
                                                 (2 << 20) + 100]))
                N.check(N.lib.glfsx_create(bs, bs, salt, None, data, len(data), sink,
                                           ctypes.byref(counts), ctypes.byref(root)))
                if bytes(root.ref) != O.create(data, bs, salt=salt)[0]:
                    errors.append((t, len(data)))
        except Exception as e:
            errors.append(e)

    th = [threading.Thread(target=worker, args=(t,)) for t in range(12)]
    [t.start() for t in th]
    [t.join() for t in th]
    assert not errors, errors[:5]


@pytest.mark.parametrize("fail_at", [1, 2, 3, 4, 5])
def test_finish_batch_store_error(gpu, O, fail_at):
    """A Writer finishing with a few staged blocks (one coalesced one-shot
    batch: 3 blocks + tail, then the index node) and a store whose
    fail_at-th Post fails: Finish returns the store error after exactly the
    reference's Posts up to the failing one, in order."""
    from glfs_amd import bigblob
    bs = 1 << 20
    data = O.fill_splitmix(3 * bs + 777, 41)
    _, _, _, want = O.create(data, bs)
    assert len(want) == 5
    log = []

    class Failing:
        def max_size(self):
            return bs

        def post(self, ct, ref, kind=0):
            log.append((kind, ref, bytes(ct)))
            if len(log) == fail_at:
                raise IOError("refused")

    w = bigblob.Machine(bs).new_writer(Failing(), None)
    w.write(data)
    with pytest.raises(bigblob.StoreError):
        w.finish()
    w.close()
    assert [(k, r, c) for k, r, c in log] == [(k, r, c) for k, r, _, c in want[:fail_at]]


def test_dropped_result_flag_fails_only_its_call(gpu, O):
    """a one-shot launch that completes without a request's
    result flag (what a launch that failed on the device leaves) fails that
    request's call with GLFSX_E_DEVICE -- and the call returns only once no
    request of it can still be launched or written, so its stack-held
    requests are never touched after it returns.  Forced with
    glfsx_debug_one_drop on a Writer's coalesced few-block post (3 blocks +
    tail = 4 requests in one call) while 12 other threads post concurrently:
    exactly that call fails, every other root equals the oracle's, and the
    poster works afterwards."""
    from glfs_amd import _native as N
    bs = 64 << 10
    data = O.fill_splitmix(3 * bs + 777, 43)
    want = O.create(data, bs)[0]
    sink = ctypes.cast(N.lib.glfsx_sink_count, N.POST_FN)

    def create(d):
        counts, root = (ctypes.c_uint64 * 2)(), N.glfsx_root()
        rc = N.lib.glfsx_create(bs, bs, None, None, d, len(d), sink, ctypes.byref(counts),
                                ctypes.byref(root))
        return rc, bytes(root.ref)

    # alone: request 1 of the call's launch loses its flag
    N.lib.glfsx_debug_one_drop(1)
    rc, _ = create(data)
    assert rc == N.GLFSX_E_DEVICE, rc
    assert b"without its result flag" in N.lib.glfsx_last_error()
    assert create(data) == (0, want)
    # among concurrent callers
    errors, fails, stop = [], [], threading.Event()

    def worker(t):
        try:
            N.check(N.lib.glfsx_set_device(0))
            rng = random.Random(300 + t)
            k = 0
            while not stop.is_set() or k < 10:
                d = rng.randbytes(rng.choice([9, 4096, 70000, 3 * bs + 5]))
                rc, r = create(d)
                if rc == N.GLFSX_E_DEVICE:
                    fails.append(t)
                elif rc != 0 or r != O.create(d, bs)[0]:
                    errors.append((t, rc, len(d)))
                k += 1
        except Exception as e:
            errors.append(e)

    th = [threading.Thread(target=worker, args=(t,)) for t in range(12)]
    [t.start() for t in th]
    N.lib.glfsx_debug_one_drop(0)
    import time
    time.sleep(0.5)
    stop.set()
    [t.join() for t in th]
    N.lib.glfsx_debug_one_drop(0xFFFFFFFF)
    assert not errors, errors[:5]
    assert len(fails) <= 1, fails
    assert create(data) == (0, want)

"""Batched PostBlob when the blob block size is below the small route's 16 KiB
(ADVICE r3): a blob longer than its block size has several data blocks and an
index node (bigblob/blob.go:120-206), so only blobs of at most
min(16 KiB, block_size) may be hashed one lane each; the rest must be
Created.  Every root is checked against the oracle's Create of the blob at
that block size with the glfs blob type salt (machine.go:50-54), through the
host batch (glfsx_post_blobs), the device batch (glfsx_post_blobs_device) and
the one-call tree route (glfsx_post_tree_device vs the three calls).
"""
import ctypes

import pytest

from test_gpu_tree_read import _tree_inputs

pytestmark = pytest.mark.gpu

LENS = [0, 1, 100, 4095, 4096, 4097, 8192, 12345, 16384, 3000, 2 * 4096 + 64]


def _want(O, salt, bs, data, offs, lens):
    return [O.create(data[o:o + ln], bs, salt=salt, closed_form=True)[0]
            for o, ln in zip(offs, lens)]


def _layout():
    offs, o = [], 0
    for ln in LENS:
        offs.append(o)
        o += ln + 16
    return offs, o


@pytest.mark.parametrize("bs", [4096, 8192, 1024])
def test_post_blobs_host_small_block_size(gpu, O, bs):
    N = gpu
    salt = O.derive_key(bytes(32), b"blob")
    offs, total = _layout()
    data = O.fill_splitmix(total, 9)
    posts = []

    @N.POST_FN
    def sink(_ctx, kind, ref, ct, n):
        posts.append((kind, ctypes.string_at(ref, 64), n, ctypes.string_at(ct, n)))
        return 0

    n = len(LENS)
    roots = ctypes.create_string_buffer(64 * n)
    N.check(N.lib.glfsx_post_blobs(bs, bs, salt, None, data, (ctypes.c_uint64 * n)(*offs),
                                   (ctypes.c_uint64 * n)(*LENS), n, sink, None, roots))
    want = _want(O, salt, bs, data, offs, LENS)
    got = [roots.raw[64 * i:64 * i + 64] for i in range(n)]
    assert got == want
    # the Posts: n sequential PostBlob calls' Post sequences
    want_posts = []
    for o, ln in zip(offs, LENS):
        want_posts += O.create(data[o:o + ln], bs, salt=salt)[3]
    assert posts == want_posts


@pytest.mark.parametrize("bs", [4096, 8192])
def test_post_blobs_device_small_block_size(gpu, O, bs):
    import numpy as np
    import torch
    N = gpu
    salt = O.derive_key(bytes(32), b"blob")
    offs, total = _layout()
    data = O.fill_splitmix(total, 10)
    d = torch.from_numpy(np.frombuffer(data + bytes(64), dtype=np.uint8).copy()).cuda()
    n = len(LENS)
    do = torch.tensor(offs, dtype=torch.int64, device="cuda")
    dl = torch.tensor(LENS, dtype=torch.int64, device="cuda")
    roots = torch.zeros(64 * n, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    N.check(N.lib.glfsx_post_blobs_device(bs, salt, None, d.data_ptr(), do.data_ptr(),
                                          dl.data_ptr(), n, 16384, None, roots.data_ptr(),
                                          None))
    torch.cuda.synchronize()
    got = bytes(roots.cpu().numpy().tobytes())
    assert [got[64 * i:64 * i + 64] for i in range(n)] == _want(O, salt, bs, data, offs, LENS)


def test_post_tree_device_small_blob_block_size(gpu, O):
    """blob_bs 4 KiB with blobs up to 16 KiB: the one-call route must give the
    oracle's blob roots and the three calls' tree root."""
    import numpy as np
    import torch
    N = gpu
    bs = 4096
    bsalt, tsalt = O.derive_key(bytes(32), b"blob"), O.derive_key(bytes(32), b"tree")
    offs, total = _layout()
    data = O.fill_splitmix(total, 12)
    d = torch.from_numpy(np.frombuffer(data + bytes(64), dtype=np.uint8).copy()).cuda()
    n = len(LENS)
    do = torch.tensor(offs, dtype=torch.int64, device="cuda")
    dl = torch.tensor(LENS, dtype=torch.int64, device="cuda")
    names = [b"f%03d" % i for i in range(n)]
    dn, dno, dm, dt, dto, _, dbs = _tree_inputs(torch, names, [b"blob"] * n, [0o644] * n, LENS,
                                                [bs] * n)
    cap = 300 * n + 4096
    roots = torch.zeros(64 * n, dtype=torch.uint8, device="cuda")
    lines = torch.zeros(cap, dtype=torch.uint8, device="cuda")
    r, t = N.glfsx_root(), ctypes.c_uint64()
    torch.cuda.synchronize()
    N.check(N.lib.glfsx_post_tree_device(n, bs, bsalt, tsalt, None, d.data_ptr(),
                                         do.data_ptr(), dl.data_ptr(), 16384, None,
                                         roots.data_ptr(), dn.data_ptr(), dno.data_ptr(),
                                         dm.data_ptr(), dt.data_ptr(), dto.data_ptr(),
                                         dbs.data_ptr(), 2 << 20, lines.data_ptr(), cap, None,
                                         ctypes.byref(r), ctypes.byref(t), None))
    torch.cuda.synchronize()
    got = bytes(roots.cpu().numpy().tobytes())
    assert [got[64 * i:64 * i + 64] for i in range(n)] == _want(O, bsalt, bs, data, offs, LENS)
    want_tree, _, _, _ = O.create(bytes(lines[:t.value].cpu().numpy().tobytes()), 2 << 20,
                                  salt=tsalt, closed_form=True)
    assert bytes(r.ref) == want_tree


def test_post_blobs_host_pipelined_groups(gpu, O):
    """glfsx_post_blobs from host memory over several 64 MiB groups: 20000
    blobs of 0..16 KiB at scattered (non-contiguous, unordered) offsets with
    larger blobs between them (one-shot medium blobs and multi-block
    Creates at bs = 2 MiB): every root and the whole Post log (kind, ref,
    ctext) equal n sequential PostBlob calls of the oracle."""
    import hashlib
    import random
    N = gpu
    bs = 2 << 20
    salt = O.derive_key(bytes(32), b"blob")
    rng = random.Random(4)
    lens = [rng.choice([0, 1, 4096, 4096, 4096, 8191, 16384, rng.randrange(16385)])
            for _ in range(20000)]
    for k in (17, 5000, 12345, 19999):
        lens[k] = rng.choice([20000, 3 * bs + 5, bs])
    order = list(range(len(lens)))
    rng.shuffle(order)                 # blob bytes laid out in another order
    offs = [0] * len(lens)
    o = 0
    for i in order:
        offs[i] = o
        o += lens[i] + rng.choice([0, 0, 3, 64])
    data = O.fill_splitmix(o + 8, 6)
    posts = []

    @N.POST_FN
    def sink(_ctx, kind, ref, ct, n):
        posts.append((kind, ctypes.string_at(ref, 64), n,
                      hashlib.sha256(ctypes.string_at(ct, n)).digest()))
        return 0

    n = len(lens)
    roots = ctypes.create_string_buffer(64 * n)
    N.check(N.lib.glfsx_post_blobs(bs, bs, salt, None, data, (ctypes.c_uint64 * n)(*offs),
                                   (ctypes.c_uint64 * n)(*lens), n, sink, None, roots))
    want_posts = []
    for i in range(n):
        r, _, _, ps = O.create(data[offs[i]:offs[i] + lens[i]], bs, salt=salt)
        assert roots.raw[64 * i:64 * i + 64] == r, i
        want_posts += [(k, ref, ln, hashlib.sha256(ct).digest()) for k, ref, ln, ct in ps]
    assert posts == want_posts


@pytest.mark.parametrize("fail_at", [1, 7, 20001])
def test_post_blobs_host_store_error_stops_in_order(gpu, O, fail_at):
    """glfsx_post_blobs from host memory with a store whose fail_at-th Post
    fails (the first group, a later one, past a multi-block blob): the call
    returns GLFSX_E_STORE and the store saw exactly the sequential PostBlob
    calls' Posts up to the failing one (blob.go:153-156: the first failing
    Post in order is returned, none after it)."""
    import hashlib
    N = gpu
    bs = 2 << 20
    salt = O.derive_key(bytes(32), b"blob")
    lens = [4096] * 20000 + [3 * bs + 5] + [4096] * 30000   # > 64 MiB of small blobs
    offs, o = [], 0
    for ln in lens:
        offs.append(o)
        o += ln
    data = O.fill_splitmix(o + 8, 17)
    log = []

    @N.POST_FN
    def sink(_ctx, kind, ref, ct, n):
        log.append((kind, ctypes.string_at(ref, 64), n, hashlib.sha256(ctypes.string_at(ct, n)).digest()))
        return 1 if len(log) == fail_at else 0

    n = len(lens)
    roots = ctypes.create_string_buffer(64 * n)
    rc = N.lib.glfsx_post_blobs(bs, bs, salt, None, data, (ctypes.c_uint64 * n)(*offs),
                                (ctypes.c_uint64 * n)(*lens), n, sink, None, roots)
    assert rc == N.GLFSX_E_STORE
    assert len(log) == fail_at
    want = []
    i = 0
    while len(want) < fail_at:
        _, _, _, ps = O.create(data[offs[i]:offs[i] + lens[i]], bs, salt=salt)
        want += [(k, r, ln, hashlib.sha256(c).digest()) for k, r, ln, c in ps]
        i += 1
    assert log == want[:fail_at]

"""The one-launch split post (k_pass_dc) must never fail silently.

A split-mode post of many workgroups runs the DEK pass and the ChaCha20+CID
pass in one launch; a CID work item waits for its block's DEK (ref.go:128-135:
the key must exist before the XOR).  Work items are taken by ticket, so a
wait only ever depends on workgroups that are already running.  The wait is
still bounded; when the bound is hit the launch is marked failed and the
calls that synchronise repeat the post with two launches.  These tests force
that (glfsx_debug_fused leaves one block's DEK unpublished) and check that
every result still equals the oracle, and run several fused launches
concurrently on different streams.
"""
import ctypes
import os
import threading

import pytest

pytestmark = pytest.mark.gpu

MIB = 1 << 20


def _torch():
    import torch
    assert torch.cuda.is_available()
    return torch


@pytest.fixture
def fused_fault():
    from glfs_amd import _native as N
    yield N.lib.glfsx_debug_fused
    N.lib.glfsx_debug_fused(0xFFFFFFFF, 0)


def _create_device(N, t, size, bs, salt=None):
    root = N.glfsx_root()
    posts = ctypes.c_uint64()
    N.check(N.lib.glfsx_create_device(bs, salt, None, t.data_ptr(), size, None,
                                      ctypes.byref(root), ctypes.byref(posts), None))
    return bytes(root.ref), posts.value


def test_fused_timeout_create_device_repeats(gpu, O, fused_fault):
    """257 MiB at 1 MiB = 257 blocks x 4 workgroups: one fused launch (a
    launch of fewer than 1024 workgroups takes the two-pass latency form,
    pass_plan).  Block 5's DEK flag is withheld; the CID items of block 5
    time out after 2 ms, the host sees the error word and repeats the Create
    with two launches: the root equals the oracle's, one failure is
    counted."""
    torch = _torch()
    from glfs_amd import _native as N
    size, bs = 256 * MIB + 4096, MIB
    t = torch.empty(size + 64, dtype=torch.uint8, device="cuda")
    N.check(N.lib.glfsx_fill_splitmix_device(t.data_ptr(), 0, size, 77, None))
    torch.cuda.synchronize()
    want, _, _, _ = O.create(O.fill_splitmix(size, 77), bs, closed_form=True)
    before = fused_fault(0xFFFFFFFF, 0)
    assert _create_device(N, t, size, bs)[0] == want       # no fault
    assert fused_fault(0xFFFFFFFF, 0) == before
    fused_fault(5, 2000)
    # the read-only counter leaves the armed fault in place
    assert N.lib.glfsx_fused_failures() == before
    assert N.lib.glfsx_fused_failures() == before
    assert _create_device(N, t, size, bs)[0] == want       # fault, repeated
    assert N.lib.glfsx_fused_failures() == before + 1
    assert fused_fault(0xFFFFFFFF, 0) == before + 1
    assert _create_device(N, t, size, bs)[0] == want       # flags/counters intact


def test_fused_timeout_post_batch_repeats(gpu, O, fused_fault):
    """glfsx_post_batch (host buffers): the faulted slab is posted again;
    every ref and ctext byte equals the oracle."""
    from glfs_amd import _native as N
    bs, total = MIB, 256 * MIB + 333       # a 256-block fused slab + 1 block
    salt = bytes(range(32))
    data = O.fill_splitmix(total, 3)
    before = fused_fault(7, 2000)
    n = (total + bs - 1) // bs
    refs = ctypes.create_string_buffer(64 * n)
    ct = ctypes.create_string_buffer(total)
    N.check(N.lib.glfsx_post_batch(salt, data, total, bs, ct, refs, None))
    assert fused_fault(0xFFFFFFFF, 0) == before + 1
    for j in (0, 6, 7, 8, n - 1):
        r, c = O.post(salt, data[j * bs:(j + 1) * bs])
        assert refs.raw[64 * j:64 * j + 64] == r, j
        assert ct.raw[j * bs:j * bs + len(c)] == c, j


def test_fused_timeout_writer_rehashes(gpu, O, fused_fault):
    """The Writer with 256-block batches (GLFSX_BATCH_MIB=256, fused
    launches): the first batch's fused launch fails; every batch in flight
    is hashed again and the Post log (kind, ref, ctext) and root equal the
    oracle writer's."""
    from glfs_amd import _native as N
    bs, total = MIB, 600 * MIB + 5
    data = O.fill_splitmix(total, 11)
    want_root, _, _, want_posts = O.create(data, bs)
    got = []

    @N.POST_FN
    def sink(_ctx, kind, ref, ct, n):
        got.append((kind, ctypes.string_at(ref, 64), n, ctypes.string_at(ct, n)))
        return 0

    old = os.environ.get("GLFSX_BATCH_MIB")
    os.environ["GLFSX_BATCH_MIB"] = "256"
    try:
        before = fused_fault(50, 2000)
        root = N.glfsx_root()
        N.check(N.lib.glfsx_create(bs, bs, None, None, data, total, sink, None,
                                   ctypes.byref(root)))
    finally:
        if old is None:
            del os.environ["GLFSX_BATCH_MIB"]
        else:
            os.environ["GLFSX_BATCH_MIB"] = old
    assert fused_fault(0xFFFFFFFF, 0) == before + 1
    assert bytes(root.ref) == want_root
    assert len(got) == len(want_posts)
    for a, b in zip(got, want_posts):
        assert a == b


def test_fused_concurrent_streams(gpu, fused_fault):
    """Three threads, each on its own stream, run config-2-shaped Creates
    (512 MiB at 2 MiB: 4096-workgroup fused launches, more than the chip
    holds at once) at the same time, five rounds: every root equals the same
    Create run alone, and no DEK wait ever times out."""
    torch = _torch()
    from glfs_amd import _native as N
    size, bs = 512 * MIB, 2 * MIB
    bufs = []
    for k in range(3):
        t = torch.empty(size + 64, dtype=torch.uint8, device="cuda")
        N.check(N.lib.glfsx_fill_splitmix_device(t.data_ptr(), 0, size, 1000 + k, None))
        bufs.append(t)
    torch.cuda.synchronize()
    alone = [_create_device(N, t, size, bs)[0] for t in bufs]
    before = fused_fault(0xFFFFFFFF, 0)
    errs, got = [], [[] for _ in bufs]

    def run(k):
        try:
            for _ in range(5):
                got[k].append(_create_device(N, bufs[k], size, bs)[0])
        except Exception as e:  # noqa: BLE001 -- reported below
            errs.append(e)

    th = [threading.Thread(target=run, args=(k,)) for k in range(3)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    assert not errs, errs
    assert fused_fault(0xFFFFFFFF, 0) == before
    for k in range(3):
        assert got[k] == [alone[k]] * 5, k

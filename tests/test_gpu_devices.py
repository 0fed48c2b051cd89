"""Multi-GPU on DISTINCT devices (BASELINE config 5), run whenever
two or more GPUs are visible and skipped with the reason otherwise (the
one-GPU rehearsals that name device 0 several times are in
test_gpu_multi.py / test_gpu_shard_mp.py).

These exercise what only a second device reaches: the Writer's device
switching (DevScope) between lanes, per-device slot / stream / scratch pools,
one-shot posts on the home device while another lane's device is current,
glfsx_create_devices' part workers on devices 1..N-1, and ranks of the
cross-process path on their own GPUs (bigblob/blob.go:120-206 split by block
ranges).  Every result is compared with the oracle or the one-device path.
"""
import ctypes
import os

import pytest

from test_gpu_multi import _create_devices, _gpu_post_log, _oracle_post_log, stream4g  # noqa
from test_gpu_shard_mp import _oracle_level1, _run_ranks

pytestmark = pytest.mark.gpu

MIB, GIB = 1 << 20, 1 << 30


def _ndev():
    import torch
    return torch.cuda.device_count()


needs2 = pytest.mark.skipif(_ndev() < 2, reason="needs >= 2 visible GPUs (distinct devices)")


@needs2
def test_writer_distinct_devices_4gib_stream(gpu, stream4g):  # noqa: F811
    """4 GiB + 12345 B in 64 MiB writes into one Writer whose batches go
    round-robin over every visible GPU: all 4097 data Posts, the index Post
    and the root equal the oracle writer's; then the lane order reversed
    (the home device last)."""
    data, (want_root, want_log) = stream4g
    devs = list(range(min(_ndev(), 8)))
    for order in (devs, devs[::-1]):
        root, log = _gpu_post_log(gpu, data, MIB, order, 64 * MIB)
        assert root == want_root
        assert log == want_log


@needs2
def test_writer_distinct_devices_fused_failure_on_home_lane(gpu, O):
    """a failed one-launch post (k_pass_dc DEK wait) in a batch
    on the home lane, completed while the other lane's device is current,
    must be seen and the batches in flight hashed again -- 256 MiB batches
    (fused launches) over lanes [0, 1], the first batch (home, device 0)
    faulted; it completes when the sixth batch (lane 1) is submitted."""
    N = gpu
    bs, total = MIB, 6 * 256 * MIB + 5
    data = O.fill_splitmix(total, 13)
    want_root, want_log = _oracle_post_log(O, data, bs)
    old = os.environ.get("GLFSX_BATCH_MIB")
    os.environ["GLFSX_BATCH_MIB"] = "256"
    try:
        before = N.lib.glfsx_debug_fused(50, 2000)
        root, log = _gpu_post_log(N, data, bs, [0, 1], 64 * MIB)
    finally:
        N.lib.glfsx_debug_fused(0xFFFFFFFF, 0)
        if old is None:
            del os.environ["GLFSX_BATCH_MIB"]
        else:
            os.environ["GLFSX_BATCH_MIB"] = old
    assert N.lib.glfsx_debug_fused(0xFFFFFFFF, 0) == before + 1
    assert root == want_root
    assert log == want_log


@needs2
def test_create_devices_distinct_ragged(gpu, O):
    """64 KiB blocks (level-1 node = 64 MiB): one part per visible GPU, each
    on its own device, part k of k+1 level-1 nodes and the last ragged; the
    root equals the one-device Create of the same bytes and the level-1 refs
    the oracle's; twice (the part workers and their pools reused)."""
    import torch
    N = gpu
    bs = 64 << 10
    span = bs * (bs // 64)
    nd = min(_ndev(), 8)
    sizes = [(k + 1) * span for k in range(nd - 1)] + [span + 5 * bs + 777]
    total = sum(sizes)
    parts, off = [], 0
    for k, s in enumerate(sizes):
        t = torch.empty(s + 64, dtype=torch.uint8, device=f"cuda:{k}")
        N.set_device(k)
        N.check(N.lib.glfsx_fill_splitmix_device(t.data_ptr(), off, s + (-s) % 8, 8, None))
        parts.append(t)
        off += s
    for k in range(nd):
        torch.cuda.synchronize(k)
    N.set_device(0)
    whole = torch.empty(total + 64, dtype=torch.uint8, device="cuda:0")
    N.check(N.lib.glfsx_fill_splitmix_device(whole.data_ptr(), 0, total + (-total) % 8, 8, None))
    torch.cuda.synchronize(0)
    want = N.glfsx_root()
    N.check(N.lib.glfsx_create_device(bs, None, None, whole.data_ptr(), total, None,
                                      ctypes.byref(want), None, None))
    n0 = -(-total // bs)
    n1 = -(-n0 // (bs // 64))
    for _ in range(2):
        root, l1, posts = _create_devices(N, bs, list(range(nd)), [t.data_ptr() for t in parts],
                                          sizes, n1)
        assert root == bytes(want.ref)
    assert l1 == _oracle_level1(O, whole[:total], bs, 0, n0)
    ms = (ctypes.c_float * (nd + 1))()
    assert N.lib.glfsx_create_devices_ms(ms, nd + 1) == nd + 1
    assert all(x >= 0 for x in ms)


@needs2
def test_create_devices_distinct_2x16gib(gpu, O):
    """Config 5's shape at two GPUs: 2 x 16 GiB at 1 MiB blocks on devices
    0 and 1, ctext written on each; root equal to the one-device Create of
    the whole 32 GiB on device 0, level-1 refs the oracle's, and sampled
    ctext blocks the oracle's."""
    import torch
    N = gpu
    bs, part = MIB, 16 * GIB
    ts, cts = [], []
    for k in range(2):
        N.set_device(k)
        t = torch.empty(part, dtype=torch.uint8, device=f"cuda:{k}")
        N.check(N.lib.glfsx_fill_splitmix_device(t.data_ptr(), k * part, part, 3, None))
        ts.append(t)
        cts.append(torch.empty(part, dtype=torch.uint8, device=f"cuda:{k}"))
    for k in range(2):
        torch.cuda.synchronize(k)
    N.set_device(0)
    root = N.glfsx_root()
    posts = ctypes.c_uint64()
    l1 = ctypes.create_string_buffer(128)
    N.check(N.lib.glfsx_create_devices(
        bs, None, None, 2, (ctypes.c_int * 2)(0, 1),
        (ctypes.c_void_p * 2)(*[t.data_ptr() for t in ts]), (ctypes.c_uint64 * 2)(part, part),
        (ctypes.c_void_p * 2)(*[c.data_ptr() for c in cts]), l1, ctypes.byref(root),
        ctypes.byref(posts)))
    assert posts.value == 32768 + 2 + 1
    want_l1 = _oracle_level1(O, ts[0], bs, 0, 16384) + _oracle_level1(O, ts[1], bs, 0, 16384)
    # _oracle_level1 of part 1 alone: blocks 0..16383 of ts[1] are blocks
    # 16384.. of the blob (same keys: a block's ref depends only on its bytes)
    assert l1.raw == want_l1
    raw = O.derive_key(bytes(32), b"raw")
    for k, j in ((0, 0), (1, 16383), (1, 77)):
        pt = bytes(ts[k][j * bs:(j + 1) * bs].cpu().numpy().tobytes())
        _, want_ct = O.post(raw, pt)
        assert bytes(cts[k][j * bs:(j + 1) * bs].cpu().numpy().tobytes()) == want_ct
    del cts
    whole = torch.empty(2 * part, dtype=torch.uint8, device="cuda:0")
    N.check(N.lib.glfsx_fill_splitmix_device(whole.data_ptr(), 0, 2 * part, 3, None))
    w = N.glfsx_root()
    N.check(N.lib.glfsx_create_device(bs, None, None, whole.data_ptr(), 2 * part, None,
                                      ctypes.byref(w), None, None))
    assert bytes(root.ref) == bytes(w.ref)


@needs2
def test_sharded_ranks_on_distinct_devices(gpu, O):
    """The cross-process path with each rank on its own GPU (rank r ->
    device r): 2 ranks over 4 level-1 nodes at 64 KiB blocks, ragged."""
    from test_gpu_shard_mp import _whole_root
    bs = 64 << 10
    total = (1024 * 4 + 5) * bs - 777
    got = _run_ranks(2, total, bs, 5, per_rank_device=True)
    want_root, t = _whole_root(total, bs, 5)
    assert got[0][3] == want_root
    for rank, (first, nb, mine, _) in got.items():
        assert mine == _oracle_level1(O, t, bs, first, nb), rank


@needs2
def test_one_shot_posts_on_each_device(gpu, O):
    """glfs.PostBlob-sized posts from one thread switching devices: each
    device's one-shot poster and salt cache give the oracle's refs."""
    N = gpu
    salt = O.derive_key(bytes(32), b"raw")
    for k in list(range(min(_ndev(), 8))) + [0]:
        N.set_device(k)
        for ln in (0, 9, 4096, 70000):
            data = O.fill_splitmix(ln, 40 + k)
            ref = ctypes.create_string_buffer(64)
            ct = ctypes.create_string_buffer(max(ln, 1))
            N.check(N.lib.glfsx_post(salt, data, ln, ct, ref, None))
            want_ref, want_ct = O.post(salt, data)
            assert ref.raw == want_ref and ct.raw[:ln] == want_ct, (k, ln)
    N.set_device(0)

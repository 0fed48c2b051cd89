"""Multi-GPU in one process (BASELINE config 5), rehearsed on one
GPU by naming device 0 several times.

* glfsx_writer_set_devices: one bigblob.Writer (blob.go:71-206) fed from one
  host stream, batches round-robin over a device list, Posts replayed in
  block order -- the Post log (kind, ref, ctext) and root must equal the
  oracle writer's for devices [0, 0] and [0, 0, 0].
* glfsx_create_devices: a device-resident blob in bf-aligned parts, each
  part's data blocks and level-1 nodes posted by its own worker, levels >= 2
  on devs[0] -- the root must equal glfsx_create_device over the whole blob
  and the level-1 refs the oracle's.
"""
import ctypes
import hashlib

import pytest

from test_gpu_shard_mp import _oracle_level1

pytestmark = pytest.mark.gpu

MIB, GIB = 1 << 20, 1 << 30


def _oracle_post_log(O, data, bs):
    """The oracle writer's (kind, ref, len, sha256(ctext)) per Post, and root."""
    L = O.lib()
    log = []

    @O.SINK_FN
    def sink(_ctx, kind, ref, ct, n):
        log.append((kind, ctypes.string_at(ref, 64), n,
                    hashlib.sha256(ctypes.string_at(ct, n)).digest()))
        return 0

    err = ctypes.c_int(0)
    w = L.oracle_writer_new(bs, bs, None, None, sink, None, ctypes.byref(err))
    assert w
    try:
        assert L.oracle_writer_write(w, data, len(data)) == 0
        root = ctypes.create_string_buffer(64)
        size, obs = ctypes.c_uint64(), ctypes.c_uint64()
        assert L.oracle_writer_finish(w, root, ctypes.byref(size), ctypes.byref(obs)) == 0
    finally:
        L.oracle_writer_free(w)
    return root.raw, log


def _gpu_post_log(N, data, bs, devs, pieces):
    log = []

    @N.POST_FN
    def sink(_ctx, kind, ref, ct, n):
        log.append((kind, ctypes.string_at(ref, 64), n,
                    hashlib.sha256(ctypes.string_at(ct, n)).digest()))
        return 0

    err = ctypes.c_int(0)
    w = N.lib.glfsx_writer_new(bs, bs, None, None, sink, None, ctypes.byref(err))
    assert w, N.last_error()
    try:
        if devs is not None:
            arr = (ctypes.c_int * len(devs))(*devs)
            N.check(N.lib.glfsx_writer_set_devices(w, arr, len(devs)))
        mv = memoryview(data)
        off = 0
        while off < len(data):
            n = min(pieces, len(data) - off)
            buf = bytes(mv[off:off + n]) if n < len(data) else data
            rc = N.lib.glfsx_writer_write(w, buf, n)
            N.check(rc, (N.lib.glfsx_writer_error(w) or b"").decode())
            off += n
        root = N.glfsx_root()
        rc = N.lib.glfsx_writer_finish(w, ctypes.byref(root))
        N.check(rc, (N.lib.glfsx_writer_error(w) or b"").decode())
    finally:
        N.lib.glfsx_writer_free(w)
    return bytes(root.ref), log


@pytest.fixture(scope="module")
def stream4g(O):
    total = 4 * GIB + 12345          # ragged tail block
    data = O.fill_splitmix(total, 21)
    return data, _oracle_post_log(O, data, MIB)


@pytest.mark.parametrize("devs", [[0, 0], [0, 0, 0]])
def test_writer_multi_device_4gib_stream(gpu, stream4g, devs):
    """4 GiB + 12345 B host stream at 1 MiB blocks into one Writer over a
    device list, in 64 MiB writes: 4097 data Posts and 1 index Post, every
    one equal to the oracle writer's, and the same root."""
    data, (want_root, want_log) = stream4g
    root, log = _gpu_post_log(gpu, data, MIB, devs, 64 * MIB)
    assert root == want_root
    assert len(log) == len(want_log)
    for i, (a, b) in enumerate(zip(log, want_log)):
        assert a == b, i


def test_writer_multi_device_small_writes(gpu, O):
    """io.Copy's 32 KiB writes (glfs.go:53) into a 3-device writer at 64 KiB
    blocks: four batches of 1024 blocks go round-robin over the devices; the
    Post log equals the oracle's."""
    bs, total = 64 << 10, (200 << 20) + 777
    data = O.fill_splitmix(total, 5)
    want_root, want_log = _oracle_post_log(O, data, bs)
    root, log = _gpu_post_log(gpu, data, bs, [0, 0, 0], 32 << 10)
    assert root == want_root
    assert log == want_log


def test_writer_set_devices_rules(gpu):
    """set_devices only before the first write; bad device ids fail; the
    device-input calls need a one-device writer."""
    N = gpu
    err = ctypes.c_int(0)
    w = N.lib.glfsx_writer_new(MIB, MIB, None, None, N.POST_FN(0), None, ctypes.byref(err))
    try:
        bad = (ctypes.c_int * 1)(9999)
        assert N.lib.glfsx_writer_set_devices(w, bad, 1) == N.GLFSX_E_ARG
        two = (ctypes.c_int * 2)(0, 0)
        assert N.lib.glfsx_writer_set_devices(w, two, 2) == 0
        assert N.lib.glfsx_writer_write_device(w, ctypes.c_void_p(16), 1, None) == \
            N.GLFSX_E_UNSUPPORTED
        w2 = N.lib.glfsx_writer_new(MIB, MIB, None, None, N.POST_FN(0), None,
                                    ctypes.byref(err))
        try:
            assert N.lib.glfsx_writer_write(w2, b"x" * 100, 100) == 0
            assert N.lib.glfsx_writer_set_devices(w2, two, 2) == N.GLFSX_E_ARG
        finally:
            N.lib.glfsx_writer_free(w2)
    finally:
        N.lib.glfsx_writer_free(w)


def _create_devices(N, bs, devs, ptrs, sizes, want_l1):
    n = len(devs)
    root = N.glfsx_root()
    posts = ctypes.c_uint64()
    l1 = ctypes.create_string_buffer(max(64 * want_l1, 1))
    N.check(N.lib.glfsx_create_devices(
        bs, None, None, n, (ctypes.c_int * n)(*devs), (ctypes.c_void_p * n)(*ptrs),
        (ctypes.c_uint64 * n)(*sizes), None, l1, ctypes.byref(root), ctypes.byref(posts)))
    return bytes(root.ref), l1.raw[:64 * want_l1], posts.value


def test_create_devices_2x16gib(gpu, O):
    """2 x 16 GiB at 1 MiB blocks on devices [0, 0]: root equal to the
    one-device Create of the whole 32 GiB blob, both level-1 refs equal to
    the threaded oracle's, 32768 + 2 + 1 Posts."""
    import torch
    N = gpu
    bs, part = MIB, 16 * GIB
    total = 2 * part
    t = torch.empty(total, dtype=torch.uint8, device="cuda")
    N.check(N.lib.glfsx_fill_splitmix_device(t.data_ptr(), 0, total, 3, None))
    torch.cuda.synchronize()
    whole = N.glfsx_root()
    N.check(N.lib.glfsx_create_device(bs, None, None, t.data_ptr(), total, None,
                                      ctypes.byref(whole), None, None))
    root, l1, posts = _create_devices(N, bs, [0, 0], [t.data_ptr(), t.data_ptr() + part],
                                      [part, part], 2)
    assert root == bytes(whole.ref)
    assert posts == 32768 + 2 + 1
    assert l1 == _oracle_level1(O, t, bs, 0, 32768)


@pytest.mark.parametrize("devs", [[0, 0, 0], [0]])
def test_create_devices_ragged_vs_oracle(gpu, O, devs):
    """64 KiB blocks (bf = 1024, level-1 node = 64 MiB): 3 parts of 1, 2 and
    1.3 level-1 nodes (the last ragged), or the whole blob as one part: root
    equal to the oracle's closed form."""
    import torch
    N = gpu
    bs = 64 << 10
    span = bs * (bs // 64)
    sizes = [span, 2 * span, span + 5 * bs + 777] if len(devs) == 3 else [4 * span + 777]
    total = sum(sizes)
    t = torch.empty(total, dtype=torch.uint8, device="cuda")
    N.check(N.lib.glfsx_fill_splitmix_device(t.data_ptr(), 0, total, 8, None))
    torch.cuda.synchronize()
    ptrs, off = [], 0
    for s in sizes:
        ptrs.append(t.data_ptr() + off)
        off += s
    n1 = -(-(-(-total // bs)) // (bs // 64))
    root, l1, _ = _create_devices(N, bs, devs, ptrs, sizes, n1)
    want, _, _, _ = O.create(t.cpu().numpy().tobytes(), bs, closed_form=True)
    assert root == want
    if len(devs) > 1:
        assert l1 == _oracle_level1(O, t, bs, 0, -(-total // bs))


def test_create_devices_rejects_unaligned_parts(gpu):
    import torch
    N = gpu
    t = torch.empty(8 * MIB, dtype=torch.uint8, device="cuda")
    root = N.glfsx_root()
    rc = N.lib.glfsx_create_devices(
        4096, None, None, 2, (ctypes.c_int * 2)(0, 0),
        (ctypes.c_void_p * 2)(t.data_ptr(), t.data_ptr() + 4 * MIB),
        (ctypes.c_uint64 * 2)(4 * MIB - 4096, 4 * MIB), None, None, ctypes.byref(root), None)
    assert rc == N.GLFSX_E_ARG


def test_create_devices_config5_level_structure(gpu, O):
    """BASELINE config 5's level structure on the one GPU (VERDICT r4 next
    #1; bigblob/blob.go:165-206): 8 parts x 16 GiB at 1 MiB blocks, device 0
    named 8 times (8 PartWorkers, each posting its 16384 data blocks and its
    one level-1 node), ctext not written -- 131072 blocks -> 8 level-1 refs
    gathered on the host -> the root node.  The root must equal
    glfsx_create_device over the same 128 GiB, the first and the last part's
    level-1 refs the oracle's, and the Posts n0 + 8 + 1."""
    import torch
    N = gpu
    bs, part, nparts = MIB, 16 * GIB, 8
    total = nparts * part
    t = torch.empty(total, dtype=torch.uint8, device="cuda")
    N.check(N.lib.glfsx_fill_splitmix_device(t.data_ptr(), 0, total, 5, None))
    torch.cuda.synchronize()
    whole, wposts = N.glfsx_root(), ctypes.c_uint64()
    N.check(N.lib.glfsx_create_device(bs, None, None, t.data_ptr(), total, None,
                                      ctypes.byref(whole), ctypes.byref(wposts), None))
    n0 = total // bs
    root, l1, posts = _create_devices(N, bs, [0] * nparts,
                                      [t.data_ptr() + k * part for k in range(nparts)],
                                      [part] * nparts, nparts)
    assert root == bytes(whole.ref)
    assert posts == n0 + nparts + 1 == wposts.value
    per = part // bs
    assert l1[:64] == _oracle_level1(O, t, bs, 0, per)
    assert l1[-64:] == _oracle_level1(O, t, bs, (nparts - 1) * per, per)
    # the gathered level-1 refs posted as the root node (blob.go:184-206)
    idx = O.derive_key(bytes(32), b"index")
    assert O.post(idx, l1.ljust(bs, b"\0"))[0] == root
    del t
    torch.cuda.empty_cache()

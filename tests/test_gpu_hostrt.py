"""BASELINE configs[2] through the host at full size: a 64 GiB blob at 1 MiB
blocks streamed from pageable host memory through the Writer (bigblob
Create, blob.go:209-217) into the pre-hashed store (keep_data off), 1024
pinned 64 MiB batches in a row.  The root must equal the device-resident
Create's root over the same bytes, the store must hold every Post, and
sampled ctexts must equal the oracle's (ref.go:98-111)."""
import ctypes
import random

import pytest

pytestmark = pytest.mark.gpu

MIB, GIB = 1 << 20, 1 << 30


def test_host_round_trip_64gib(gpu, O):
    import torch
    N = gpu
    bs, size, seed = MIB, 64 * GIB, 3
    t = torch.empty(size, dtype=torch.uint8, device="cuda")
    N.check(N.lib.glfsx_fill_splitmix_device(t.data_ptr(), 0, size, seed, None))
    torch.cuda.synchronize()
    want = N.glfsx_root()
    N.check(N.lib.glfsx_create_device(bs, None, None, t.data_ptr(), size, None,
                                      ctypes.byref(want), None, None))
    host = t.cpu().numpy()            # pageable, 64 GiB
    del t
    torch.cuda.empty_cache()
    n0 = size // bs
    rng = random.Random(64)
    sample = sorted({0, 1, n0 - 1} | set(rng.sample(range(n0), 5)))
    store = N.lib.glfsx_store_new(bs, N.GLFSX_STORE_TRUST, 0, 0, None)
    assert store
    store_post = ctypes.cast(N.lib.glfsx_store_post, N.POST_FN)
    seen = {"data": 0, "index": 0}
    got = {}

    @N.POST_FN
    def sink(_ctx, kind, ref, ct, n):
        if kind == 0:
            b = seen["data"]
            seen["data"] += 1
            if b in sample:
                got[b] = (ctypes.string_at(ref, 64), ctypes.string_at(ct, n))
        else:
            seen["index"] += 1
        return store_post(ctypes.c_void_p(store), kind, ref, ct, n)

    try:
        root = N.glfsx_root()
        N.check(N.lib.glfsx_create(bs, bs, None, None, host.ctypes.data, size, sink, None,
                                   ctypes.byref(root)))
        posts = ctypes.c_uint64()
        nblobs = N.lib.glfsx_store_stats(ctypes.c_void_p(store), ctypes.byref(posts), None, None)
    finally:
        N.lib.glfsx_store_free(store)
    assert bytes(root.ref) == bytes(want.ref)
    assert root.size == size and root.block_size == bs
    assert seen == {"data": n0, "index": 4 + 1}
    assert posts.value == n0 + 5 and nblobs == n0 + 5
    raw = O.derive_key(bytes(32), b"raw")
    for b in sample:
        r, c = O.post(raw, host[b * bs:(b + 1) * bs].tobytes())
        assert got[b] == (r, c), b

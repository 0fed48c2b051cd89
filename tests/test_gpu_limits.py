"""Block sizes past one workgroup's reach and the split-mode merge.

bigblob accepts any blockSize <= the store's MaxSize (blob.go:85-95); blocks
above 256 lanes x 64 chunks (16 MiB) always span several workgroups, whose
subtree CVs the message's last-arriving workgroup merges (agent-scope
release/acquire across XCDs, per-message arrival counters that every launch
leaves at zero).  Every result is compared with the oracle."""
import ctypes
import random

import pytest

pytestmark = pytest.mark.gpu

MIB = 1 << 20


def _torch():
    import torch
    return torch


def _dev(torch, n, seed):
    from glfs_amd import _native as N
    t = torch.empty(max(n, 1) + 64, dtype=torch.uint8, device="cuda")
    N.check(N.lib.glfsx_fill_splitmix_device(t.data_ptr(), 0, n, seed, None))
    torch.cuda.synchronize()
    return t


def _host(t, n):
    return bytes(t[:n].cpu().numpy().tobytes())


def _oracle_refs(O, salt, data, bs):
    L = O.lib()
    n = -(-len(data) // bs)
    out = ctypes.create_string_buffer(64 * n)
    L.oracle_post_batch(out, None, salt, data, len(data), bs, None, 16)
    return out.raw


@pytest.mark.parametrize("bs", [32 * MIB, 64 * MIB])
def test_block_size_above_16mib(gpu, O, bs):
    """Create (Writer from host memory and device-resident) at 32 / 64 MiB
    blocks: 2 full blocks and a ragged tail, every Post and the root."""
    torch = _torch()
    from glfs_amd import _native as N, bigblob
    size = 2 * bs + 12345
    t = _dev(torch, size, 41)
    data = _host(t, size)
    want_root, _, _, want_posts = O.create(data, bs)
    st = bigblob.MemStore(bs)
    root = bigblob.Machine(bs).create(st, None, data)
    assert root.ref.marshal_binary() == want_root
    assert [(k, r) for k, r, _ in st.log] == [(k, r) for k, r, _, _ in want_posts]
    r = N.glfsx_root()
    np_ = ctypes.c_uint64()
    N.check(N.lib.glfsx_create_device(bs, None, None, t.data_ptr(), size, None,
                                      ctypes.byref(r), ctypes.byref(np_), None))
    assert bytes(r.ref) == want_root and np_.value == len(want_posts)
    # DeriveKey over more than 16 MiB (ref.go:152)
    assert bigblob.derive_key(bytes(range(32)), data[:bs + 7]) == \
        O.derive_key(bytes(range(32)), data[:bs + 7])


def test_split_merge_repeated_launches(gpu, O):
    """Split launches of different shapes back to back on one stream (the
    arrival counters must return to zero after each), every message split
    over many workgroups spread over all XCDs; all refs vs the oracle."""
    torch = _torch()
    from glfs_amd import _native as N
    salt = O.derive_key(bytes(32), b"raw")
    prev = N.set_split_target(1 << 20)          # maximal split
    try:
        t = _dev(torch, 96 * MIB + 777, 5)
        data = _host(t, 96 * MIB + 777)
        rng = random.Random(3)
        shapes = [(2 * MIB, 37 * 2 * MIB + 5), (1 * MIB, 96 * MIB + 777),
                  (4 * MIB, 4 * MIB), (2 * MIB, 2 * MIB * 3), (256 * 1024, 19 * MIB + 1)]
        for rep in range(2):
            for bs, total in shapes:
                n = -(-total // bs)
                refs = torch.zeros(64 * n, dtype=torch.uint8, device="cuda")
                N.check(N.lib.glfsx_post_batch_device(salt, t.data_ptr(), total, bs, None,
                                                      refs.data_ptr(), None, None))
                torch.cuda.synchronize()
                assert _host(refs, 64 * n) == _oracle_refs(O, salt, data[:total], bs), (rep, bs)
        # the default split target again, and a random mix of sizes
        N.set_split_target(prev)
        for _ in range(3):
            bs = rng.choice([MIB, 2 * MIB, 8 * MIB])
            total = rng.randrange(1, 90 * MIB)
            n = -(-total // bs)
            refs = torch.zeros(64 * n, dtype=torch.uint8, device="cuda")
            N.check(N.lib.glfsx_post_batch_device(salt, t.data_ptr(), total, bs, None,
                                                  refs.data_ptr(), None, None))
            torch.cuda.synchronize()
            assert _host(refs, 64 * n) == _oracle_refs(O, salt, data[:total], bs), (bs, total)
    finally:
        N.set_split_target(prev)


def test_index_levels_split_quad(gpu, O):
    """Index-node passes (k_quad, split over workgroups, merged by the last
    one) at 1 / 2 / 8 MiB nodes: create_device roots vs the oracle."""
    torch = _torch()
    from glfs_amd import _native as N
    for bs, nblk in [(MIB, 3), (2 * MIB, 5), (8 * MIB, 2)]:
        size = bs * nblk + 99
        t = _dev(torch, size, bs)
        r = N.glfsx_root()
        N.check(N.lib.glfsx_create_device(bs, None, None, t.data_ptr(), size, None,
                                          ctypes.byref(r), None, None))
        assert bytes(r.ref) == O.create(_host(t, size), bs, closed_form=True)[0], bs

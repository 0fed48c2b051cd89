"""Parity of the HIP path (through the C-ABI) with the CPU oracle.

Bit-exact on every byte: refs (CID || DEK), ctext, Post order, roots.
Sizes where the oracle finishes in seconds are compared directly; the 1 GiB
config-2 blob is compared block by block with the threaded oracle; larger
device-resident blobs are checked through size-independent properties
(determinism, in-place == out-of-place, shard/gather == whole, sampled blocks
against the oracle, decrypt round trip).
"""
import ctypes
import json
import os
import random
import threading

import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
KIB, MIB, GIB = 1 << 10, 1 << 20, 1 << 30


def _torch():
    import torch
    assert torch.cuda.is_available()
    return torch


def dev_bytes(torch, n, seed=None, data=None):
    t = torch.empty(max(n, 1) + 64, dtype=torch.uint8, device="cuda")
    if data is not None:
        t[:n].copy_(torch.frombuffer(bytearray(data), dtype=torch.uint8) if n else t[:0])
    elif seed is not None:
        from glfs_amd import _native as N
        N.check(N.lib.glfsx_fill_splitmix_device(t.data_ptr(), 0, n, seed, None))
    # torch works on its own stream, glfsx on a per-thread stream: order them
    torch.cuda.synchronize()
    return t


def zeros(torch, n):
    t = torch.zeros(n, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    return t


def host(t, n):
    return bytes(t[:n].cpu().numpy().tobytes())


# ---------------------------------------------------------------- primitives
def test_fill_matches_oracle(gpu, O):
    torch = _torch()
    for n, seed in [(1, 1), (7, 2), (8, 3), (1000, 4), (1 << 20, 5)]:
        t = dev_bytes(torch, n, seed=seed)
        torch.cuda.synchronize()
        assert host(t, n) == O.fill_splitmix(n, seed)


def test_derive_key(gpu, O):
    from glfs_amd import bigblob
    rng = random.Random(1)
    salts = [bytes(32), bytes(range(32)), bytes(rng.randrange(256) for _ in range(32))]
    sizes = [0, 1, 3, 5, 63, 64, 65, 1023, 1024, 1025, 2048, 3000, 4096, 5000,
             65536, 262144 + 1, 1 << 20, (2 << 20) + 7]
    for salt in salts:
        for n in sizes:
            data = O.fill_splitmix(n, n + 1)
            assert bigblob.derive_key(salt, data) == O.derive_key(salt, data), n
    assert bigblob.derive_key(bytes(32), b"raw", 16) == O.derive_key(bytes(32), b"raw")[:16]


def test_crypto_xor(gpu, O):
    from glfs_amd import bigblob
    for n in [0, 1, 63, 64, 65, 1000, 4096, 1 << 20]:
        key = O.fill_splitmix(32, n)
        data = O.fill_splitmix(n, n + 9)
        assert bigblob.crypto_xor(key, data) == O.chacha20_xor(data, key)


def _post_batch_host(salt, data, bs, cid_key=None):
    from glfs_amd import _native as N
    n = (len(data) + bs - 1) // bs
    refs = ctypes.create_string_buffer(max(64 * n, 1))
    ct = ctypes.create_string_buffer(max(len(data), 1))
    N.check(N.lib.glfsx_post_batch(salt, data, len(data), bs, ct, refs, cid_key))
    return refs.raw[:64 * n], ct.raw[:len(data)]


@pytest.mark.parametrize("bs", [128, 1000, 1024, 4096, 65536, 300_000, 1 << 20,
                                2 << 20, 5 << 20])
def test_post_batch_vs_oracle(gpu, O, bs):
    rng = random.Random(bs)
    salt = bytes(rng.randrange(256) for _ in range(32))
    for total in sorted({1, bs - 1, bs, bs + 1, 3 * bs + rng.randrange(1, bs),
                         min(8 * bs, 12 << 20)}):
        data = O.fill_splitmix(total, total)
        refs, ct = _post_batch_host(salt, data, bs)
        for j in range(0, (total + bs - 1) // bs):
            blk = data[j * bs:(j + 1) * bs]
            r, c = O.post(salt, blk)
            assert refs[64 * j:64 * j + 64] == r, (bs, total, j)
            assert ct[j * bs:j * bs + len(blk)] == c, (bs, total, j)


@pytest.fixture
def split_target():
    """Restores the split-mode target (include/glfsx.h) after a test."""
    from glfs_amd import _native as N
    old = N.set_split_target(2048)
    N.set_split_target(old)
    yield N.set_split_target
    N.set_split_target(old)


@pytest.fixture
def latency_wgs():
    """Restores the latency-mode threshold (include/glfsx.h) after a test."""
    from glfs_amd import _native as N
    old = N.set_latency_wgs(512)
    N.set_latency_wgs(old)
    yield N.set_latency_wgs
    N.set_latency_wgs(old)


@pytest.mark.parametrize("bs,total", [(1 << 20, (40 << 20) + 77), (65536, 65536 * 600 + 1),
                                      (4096, 4096 * 3000 + 5), (2 << 20, 2 << 20)])
def test_arx_forms_vs_oracle(gpu, O, latency_wgs, split_target, bs, total):
    """Both ARX forms (asm-form kernels for many workgroups, compiler form +
    split CID pass in latency mode) on the same inputs: refs, ctext, the
    read-side decrypt and small-blob roots bit-exact with each other and the
    oracle.  Threshold 0 = never latency mode, 2**31 = always."""
    torch = _torch()
    from glfs_amd import _native as N, bigblob, glfs
    rng = random.Random(total)
    salt = bytes(rng.randrange(256) for _ in range(32))
    data = O.fill_splitmix(total, total + 11)
    blobs = [O.fill_splitmix(n, 7000 + i) for i, n in
             enumerate([4096] * 300 + [0, 1, 1000, 5000, 16384])]
    outs, decs, smalls = [], [], []
    for thr in (0, 1 << 31):
        latency_wgs(thr)
        for target in (0, 2048):
            split_target(target)
            refs, ct = _post_batch_host(salt, data, bs)
            outs.append((refs, ct))
            n0 = (total + bs - 1) // bs
            assert len(refs) == 64 * n0
            # read side (getF, batched): back to the plaintext
            ctd, refd = dev_bytes(torch, total, data=ct), dev_bytes(torch, len(refs), data=refs)
            pt = zeros(torch, total + 64)
            N.check(N.lib.glfsx_decrypt_batch_device(ctd.data_ptr(), total, bs,
                                                     refd.data_ptr(), pt.data_ptr(), None))
            torch.cuda.synchronize()
            decs.append(host(pt, total))
        smalls.append([r.root.ref.marshal_binary() for r in
                       glfs.Machine().post_blobs(bigblob.MemStore(2 << 20), blobs)])
    assert all(o == outs[0] for o in outs)
    assert all(d == data for d in decs)
    assert smalls[0] == smalls[1]
    refs, ct = outs[0]
    n0 = (total + bs - 1) // bs
    for j in sorted({0, n0 - 1} | set(rng.sample(range(n0), min(3, n0)))):
        blk = data[j * bs:(j + 1) * bs]
        r, c = O.post(salt, blk)
        assert refs[64 * j:64 * j + 64] == r, j
        assert ct[j * bs:j * bs + len(blk)] == c, j
    blob_salt = O.derive_key(bytes(32), b"blob")
    for i in (0, 299, 300, 301, 302, 303, 304):
        want, _, _, _ = O.create(blobs[i], 2 << 20, salt=blob_salt)
        assert smalls[0][i] == want, i


@pytest.mark.parametrize("bs,total", [(2 << 20, (37 << 20) + 123), (1 << 20, (70 << 20) + 1),
                                      (300_000, 300_000 * 700 + 77), (4 << 20, 24 << 20)])
def test_fused_split_post_vs_oracle(gpu, O, latency_wgs, split_target, bs, total):
    """Split-mode posts of many workgroups run both passes in one launch
    (k_pass_dc: DEK workgroups publish each message's DEK with a ready flag,
    CID workgroups of the same launch wait for it).  Every ref and ctext
    byte vs the oracle, keyed and unkeyed CIDs, at the default split target
    and at maximal split (one chunk per lane), ragged last blocks, repeated
    launches (the flags carry a per-launch epoch)."""
    rng = random.Random(bs + total)
    salt = bytes(rng.randrange(256) for _ in range(32))
    data = O.fill_splitmix(total, total + 5)
    latency_wgs(0)          # many-wave kernels even for small launches
    n0 = (total + bs - 1) // bs
    want = [O.post(salt, data[j * bs:(j + 1) * bs]) for j in range(n0)]
    for target in (2048, 1 << 31, 2048):
        split_target(target)
        refs, ct = _post_batch_host(salt, data, bs)
        for j, (r, c) in enumerate(want):
            assert refs[64 * j:64 * j + 64] == r, (target, j)
            assert ct[j * bs:j * bs + len(c)] == c, (target, j)
    split_target(2048)
    ck = bytes(range(32))
    refs, _ = _post_batch_host(salt, data, bs, cid_key=ck)
    for j in sorted({0, n0 - 1, rng.randrange(n0)}):
        assert refs[64 * j:64 * j + 64] == O.post(salt, data[j * bs:(j + 1) * bs],
                                                  cid_key=ck)[0], j


@pytest.mark.parametrize("bs,total", [(1 << 20, (3 << 20) + 5), (1 << 20, 9 << 20),
                                      (2 << 20, (5 << 20) + 999), (5 << 20, 11 << 20),
                                      (300_000, 2_000_003), (65536, 65536 * 3 + 1),
                                      (1024, 5000), (16 << 20, (16 << 20) + 1)])
def test_split_modes_vs_oracle(gpu, O, split_target, bs, total):
    """Split mode (several workgroups per block + merge launch) vs one
    workgroup per block vs the oracle: refs and ctext bit-exact.  Targets:
    0 = never split, 2048 = default, 2**31 = split every block maximally."""
    rng = random.Random(bs ^ total)
    salt = bytes(rng.randrange(256) for _ in range(32))
    data = O.fill_splitmix(total, total + 3)
    outs = []
    for target in (0, 2048, 1 << 31):
        split_target(target)
        outs.append(_post_batch_host(salt, data, bs))
        outs.append(_post_batch_host(salt, data, bs, cid_key=bytes(range(32))))
    assert outs[0] == outs[2] == outs[4]
    assert outs[1] == outs[3] == outs[5]
    refs, ct = outs[0]
    for j in range(0, (total + bs - 1) // bs):
        blk = data[j * bs:(j + 1) * bs]
        r, c = O.post(salt, blk)
        assert refs[64 * j:64 * j + 64] == r, (bs, total, j)
        assert ct[j * bs:j * bs + len(blk)] == c, (bs, total, j)
    j = rng.randrange((total + bs - 1) // bs)
    r, _ = O.post(salt, data[j * bs:(j + 1) * bs], cid_key=bytes(range(32)))
    assert outs[1][0][64 * j:64 * j + 64] == r


def test_split_modes_create_device(gpu, O, split_target):
    """Index levels in split mode: a 3-level tree at 4 KiB blocks and a
    17-block blob at 1 MiB, roots equal across targets and to the oracle."""
    torch = _torch()
    for bs, size in [(4096, 4096 * 64 * 2 + 7), (1 << 20, (17 << 20) + 5)]:
        t = dev_bytes(torch, size, seed=size)
        roots = set()
        for target in (0, 2048, 1 << 31):
            split_target(target)
            roots.add(_create_device(torch, bs, t, size))
        assert len(roots) == 1
        want, _, _, want_posts = O.create(O.fill_splitmix(size, size), bs, salt=None,
                                          closed_form=True)
        root, posts = roots.pop()
        assert root == want and posts == len(want_posts)


def test_post_batch_keyed_cid(gpu, O):
    key = bytes(range(100, 132))
    data = O.fill_splitmix(5 * 4096 + 17, 11)
    refs, ct = _post_batch_host(bytes(32), data, 4096, cid_key=key)
    for j in range(6):
        r, c = O.post(bytes(32), data[j * 4096:(j + 1) * 4096], cid_key=key)
        assert refs[64 * j:64 * j + 64] == r


def test_unaligned_device_pointers(gpu, O):
    """The byte-load kernel variant (src/ctext not 16-B aligned)."""
    torch = _torch()
    from glfs_amd import _native as N
    bs, total = 4096, 3 * 4096 + 100
    data = O.fill_splitmix(total, 21)
    for off in (1, 2, 3, 4, 8):
        buf = dev_bytes(torch, total + off, data=bytes(off) + data)
        ctb = zeros(torch, total + 64)
        refs = zeros(torch, 64 * 4)
        N.check(N.lib.glfsx_post_batch_device(bytes(32), buf.data_ptr() + off, total, bs,
                                              ctb.data_ptr() + 3, refs.data_ptr(), None,
                                              None))
        torch.cuda.synchronize()
        rh, ch = host(refs, 256), host(ctb, total + 3)[3:]
        for j in range(4):
            r, c = O.post(bytes(32), data[j * bs:(j + 1) * bs])
            assert rh[64 * j:64 * j + 64] == r, (off, j)
            assert ch[j * bs:j * bs + len(c)] == c


# ------------------------------------------------------------ bigblob writer
GOLDEN = json.load(open(os.path.join(HERE, "golden", "bigblob.json")))


def _data(O, gen, n):
    if gen == "mod251":
        return O.mod251(n)
    if gen.startswith("splitmix:"):
        return O.fill_splitmix(n, int(gen.split(":")[1]))
    return gen.split(":", 1)[1].encode()


@pytest.mark.parametrize("c", GOLDEN["cases"], ids=lambda c: c["name"])
def test_golden_vectors(gpu, O, c):
    from glfs_amd import bigblob
    data = _data(O, c["gen"], c["size"])
    salt = bytes.fromhex(c["salt"]) if c["salt"] else None
    store = bigblob.MemStore(c["block_size"])
    root = bigblob.Machine(c["block_size"]).create(store, salt, data)
    assert root.ref.cid.hex() == c["root"]["cid"]
    assert root.ref.dek.hex() == c["root"]["dek"]
    assert (root.size, root.block_size) == (c["root"]["size"], c["root"]["blockSize"])
    assert len(store.log) == c["n_posts"]
    if "posts" in c:
        got = [[k, n, r[:32].hex(), r[32:].hex()] for k, r, n in store.log]
        assert got == c["posts"]
    # every stored ctext hashes to its CID (the store's own check, ref.go:103)
    for cid, ct in list(store.blobs.items())[:64]:
        assert O.blake3(ct) == cid
    # read side round trip (blob.go:31-69, ref.go:113-126)
    if c["block_size"] % 64 == 0 and c["size"] <= (4 << 20) + 1:
        assert bigblob.read_all(store, root) == data


def test_glfs_config1(gpu):
    """examples/write-read-blob: glfs.PostBlob("test data").  With the 1 MiB
    store of the example the reference panics at HEAD (blob.go:90-92); with a
    2 MiB store the ref is SURVEY's anchor."""
    from glfs_amd import _native as N, bigblob, glfs
    with pytest.raises(N.Panic, match="2097152 > maxSize 1048576"):
        glfs.post_blob(bigblob.MemStore(1 << 20), b"test data")
    s = bigblob.MemStore(2 << 20)
    ref = glfs.post_blob(s, b"test data")
    assert ref.type == "blob"
    assert ref.root.ref.cid.hex() == \
        "c46ac4e44a328b9c07cba45eddb89b635fa44746823f4f5d3f01e39f52a6c851"
    assert ref.root.ref.dek.hex() == \
        "d0d02185d4646a367978c907c9b04fd4b7c536467d9c1882a67b2079b8c9841d"
    assert (ref.root.size, ref.root.block_size) == (9, 2 << 20)
    assert bigblob.read_all(s, ref.root) == b"test data"


def test_writer_streaming_vs_oracle(gpu, O):
    """Random write granularity; the full Post sequence (kind, ref, ctext) must
    equal the reference writer's (blob.go:120-206)."""
    from glfs_amd import bigblob
    rng = random.Random(3)
    for bs, size in [(1024, 70_000), (4096, 4096 * 64 * 2 + 5), (128, 20_000),
                     (1 << 20, 5 * (1 << 20) + 3)]:
        data = O.fill_splitmix(size, bs)
        pieces, left = [], size
        while left:
            k = min(left, rng.choice([1, 13, bs - 1, bs, bs + 1, 5 * bs + 7, 100_000]))
            pieces.append(k)
            left -= k
        want_root, _, _, want_posts = O.create(data, bs, salt=None, chunks=pieces)
        store = bigblob.MemStore(bs)
        w = bigblob.Machine(bs).new_writer(store)
        off = 0
        for k in pieces:
            w.write(data[off:off + k])
            off += k
        root = w.finish()
        w.close()
        assert root.ref.marshal_binary() == want_root
        assert [(k, r) for k, r, _ in store.log] == [(k, r) for k, r, _, _ in want_posts]
        for k, r, _, ct in want_posts:
            assert store.blobs[r[:32]] == ct


def test_store_error_surfaces(gpu, O):
    from glfs_amd import _native as N, bigblob

    class Flaky(bigblob.MemStore):
        def post(self, ctext, ref, kind=0):
            if len(self.log) == 2:
                raise IOError("disk full")
            super().post(ctext, ref, kind)

    with pytest.raises(N.StoreError):
        bigblob.Machine(1024).create(Flaky(1024), None, O.fill_splitmix(10_000, 1))


def test_concurrent_writers(gpu, O):
    """glfs.Machine is used concurrently (machine.go:25): per-thread streams."""
    from glfs_amd import bigblob
    results = {}

    def work(i):
        data = O.fill_splitmix(50_000 + 997 * i, 100 + i)
        root = bigblob.Machine(4096).create(bigblob.MemStore(4096), None, data)
        results[i] = (root.ref.marshal_binary(), data)

    ts = [threading.Thread(target=work, args=(i,)) for i in range(6)]
    [t.start() for t in ts]
    [t.join() for t in ts]
    for i, (got, data) in results.items():
        assert got == O.create(data, 4096, salt=None)[0]


# ------------------------------------------------------ device-resident path
def _create_device(torch, bs, t, size, ctext=None, salt=None):
    from glfs_amd import _native as N
    r = N.glfsx_root()
    posts = ctypes.c_uint64()
    N.check(N.lib.glfsx_create_device(bs, salt, None, t.data_ptr(), size,
                                      ctext.data_ptr() if ctext is not None else None,
                                      ctypes.byref(r), ctypes.byref(posts), None))
    return bytes(r.ref), posts.value


@pytest.mark.parametrize("bs,size", [(1 << 20, 0), (1 << 20, 1), (1 << 20, 1 << 20),
                                     (1 << 20, (17 << 20) + 5), (2 << 20, 64 << 20),
                                     (1024, 16 * 1024 * 16 + 1), (4096, 3 << 20)])
def test_create_device_vs_oracle(gpu, O, bs, size):
    torch = _torch()
    seed = size + bs
    t = dev_bytes(torch, size, seed=seed)
    ct = torch.empty(size + 64, dtype=torch.uint8, device="cuda")
    root, posts = _create_device(torch, bs, t, size, ct)
    data = O.fill_splitmix(size, seed)
    want, _, _, want_posts = O.create(data, bs, salt=None, closed_form=True)
    assert root == want
    assert posts == len(want_posts)
    got_ct = host(ct, size)
    for j in range((size + bs - 1) // bs):
        blk = data[j * bs:(j + 1) * bs]
        _, c = O.post(O.derive_key(bytes(32), b"raw"), blk)
        assert got_ct[j * bs:j * bs + len(blk)] == c, j


def test_shard_gather_equals_whole(gpu, O):
    """disjoint block ranges aligned to bf, level-1 refs gathered,
    root built from them == root of the whole blob == oracle."""
    torch = _torch()
    from glfs_amd import _native as N
    bs = 4096
    bf = bs // 64
    size = bs * (bf * 5 + 3) + 777
    n0 = (size + bs - 1) // bs
    t = dev_bytes(torch, size, seed=77)
    whole, _ = _create_device(torch, bs, t, size)
    want = O.create(O.fill_splitmix(size, 77), bs, salt=None, closed_form=True)[0]
    assert whole == want
    for shards in (2, 3, 6):
        per = -(-n0 // shards)
        per = -(-per // bf) * bf
        level1 = b""
        for b0 in range(0, n0, per):
            nb = min(per, n0 - b0)
            out = ctypes.create_string_buffer(64 * (-(-nb // bf)))
            N.check(N.lib.glfsx_shard_device(bs, None, None, t.data_ptr() + b0 * bs, size,
                                             b0, nb, None, out, None))
            level1 += out.raw
        r = N.glfsx_root()
        N.check(N.lib.glfsx_root_from_level1(bs, None, None, level1, len(level1) // 64,
                                             size, ctypes.byref(r)))
        assert bytes(r.ref) == whole, shards


def test_config2_1gib_2mib(gpu, O):
    """BASELINE config 2: 1 GiB at the glfs default 2 MiB block size
    (splitmix seed 1): every one of the 512 data refs and the root, bit-exact."""
    torch = _torch()
    from glfs_amd import _native as N
    size, bs = GIB, 2 << 20
    n0 = size // bs
    blob_salt = O.derive_key(bytes(32), b"blob")
    raw = O.derive_key(blob_salt, b"raw")
    idx = O.derive_key(blob_salt, b"index")
    t = dev_bytes(torch, size, seed=1)
    refs = zeros(torch, 64 * n0)
    N.check(N.lib.glfsx_post_batch_device(raw, t.data_ptr(), size, bs, None,
                                          refs.data_ptr(), None, None))
    root, posts = _create_device(torch, bs, t, size, salt=blob_salt)
    torch.cuda.synchronize()
    got = host(refs, 64 * n0)
    L = O.lib()
    data = ctypes.create_string_buffer(size)
    L.oracle_fill_splitmix(data, 0, size, 1)
    want = ctypes.create_string_buffer(64 * n0)
    L.oracle_post_batch(want, None, raw, data, size, bs, None, 16)
    assert got == want.raw
    node = want.raw + bytes(bs - 64 * n0)
    r_root, _ = O.post(idx, node)
    assert root == r_root
    assert posts == n0 + 1


def test_large_blob_properties(gpu, O):
    """4 GiB at 1 MiB, device-resident: determinism, in-place == out-of-place,
    sampled blocks vs oracle, decrypt of sampled ctext blocks."""
    torch = _torch()
    from glfs_amd import _native as N, bigblob
    size, bs = 4 * GIB, MIB
    n0 = size // bs
    raw = O.derive_key(bytes(32), b"raw")
    t = dev_bytes(torch, size, seed=123)
    ct = torch.empty(size, dtype=torch.uint8, device="cuda")
    r1, p1 = _create_device(torch, bs, t, size, ct)
    r2, p2 = _create_device(torch, bs, t, size)
    assert r1 == r2 and p1 == p2 == n0 + 1  # n0 < bf: one index node
    refs = zeros(torch, 64 * n0)
    N.check(N.lib.glfsx_post_batch_device(raw, t.data_ptr(), size, bs, None,
                                          refs.data_ptr(), None, None))
    torch.cuda.synchronize()
    rh = host(refs, 64 * n0)
    rng = random.Random(9)
    for j in [0, 1, n0 - 1] + rng.sample(range(n0), 6):
        blk = host(t[j * bs:], bs)
        r, c = O.post(raw, blk)
        assert rh[64 * j:64 * j + 64] == r, j
        cth = host(ct[j * bs:], bs)
        assert cth == c
        assert bigblob.crypto_xor(r[32:], cth) == blk
    # in place: ctext over ptext gives the same refs
    N.check(N.lib.glfsx_post_batch_device(raw, t.data_ptr(), size, bs, t.data_ptr(),
                                          refs.data_ptr(), None, None))
    torch.cuda.synchronize()
    assert host(refs, 64 * n0) == rh


def test_config3_64gib_every_ref(gpu, O):
    """BASELINE config 3 at its full size (the bench workload): a 64 GiB
    device-resident blob at 1 MiB blocks, splitmix seed 3.  Every one of the
    65536 data refs and every ctext byte against the threaded oracle (1 GiB
    at a time, ptext copied down from HBM), then the two index levels and
    the root rebuilt by the oracle from those refs (blob.go:165-206)."""
    torch = _torch()
    import numpy as np
    from glfs_amd import _native as N
    size, bs, seed = 64 * GIB, MIB, 3
    n0, bf = size // bs, bs // 64
    raw = O.derive_key(bytes(32), b"raw")
    idx = O.derive_key(bytes(32), b"index")
    # a card that cannot hold it is a skip; a card that can but has the HBM
    # held elsewhere is a failure, never a silent skip
    torch.cuda.empty_cache()
    free, total = torch.cuda.mem_get_info()
    if total < 2 * size + GIB:
        pytest.skip(f"needs {2 * size + GIB} B of HBM, the device has {total}")
    assert free >= 2 * size + GIB, f"needs {2 * size + GIB} B of HBM, only {free} free"
    t = dev_bytes(torch, size, seed=seed)
    ct = torch.empty(size, dtype=torch.uint8, device="cuda")
    root, posts = _create_device(torch, bs, t, size, ct)
    refs = zeros(torch, 64 * n0)
    N.check(N.lib.glfsx_post_batch_device(raw, t.data_ptr(), size, bs, None,
                                          refs.data_ptr(), None, None))
    torch.cuda.synchronize()
    got_refs = host(refs, 64 * n0)
    L = O.lib()
    piece = GIB
    want_refs = np.empty(64 * (piece // bs), dtype=np.uint8)
    want_ct = np.empty(piece, dtype=np.uint8)
    for off in range(0, size, piece):
        pt = t[off:off + piece].cpu().numpy()
        L.oracle_post_batch(want_refs.ctypes.data, want_ct.ctypes.data, raw,
                            pt.ctypes.data, piece, bs, None, 16)
        j0 = off // bs
        assert got_refs[64 * j0:64 * (j0 + piece // bs)] == want_refs.tobytes(), off
        assert np.array_equal(ct[off:off + piece].cpu().numpy(), want_ct), off
    del t, ct
    torch.cuda.empty_cache()
    level = got_refs
    while len(level) > 64:
        level = b"".join(O.post(idx, level[i:i + bs].ljust(bs, b"\0"))[0]
                         for i in range(0, len(level), 64 * bf))
    assert root == level
    assert posts == n0 + 4 + 1
    # the root bench.py prints for this workload
    assert root[:32].hex().startswith("e87d3dc4ad171bce")


# ------------------------------------------------------------- small blobs
def test_post_blobs_vs_oracle(gpu, O):
    """Batched glfs.PostBlob (config 4 shape): every root, every Post, in order,
    equal to n sequential reference PostBlob calls; empty and ragged blobs,
    packed at unaligned offsets."""
    from glfs_amd import bigblob, glfs
    rng = random.Random(11)
    blob_salt = O.derive_key(bytes(32), b"blob")
    lens = [0, 1, 9, 63, 64, 65, 1023, 1024, 1025, 4095, 4096, 4097, 8192, 16384]
    lens += [rng.randrange(0, 16385) for _ in range(200)] + [4096] * 300
    blobs = [O.fill_splitmix(n, 1000 + i) for i, n in enumerate(lens)]
    store = bigblob.MemStore(2 << 20)
    refs = glfs.Machine().post_blobs(store, blobs)
    assert len(store.log) == len(blobs)
    for i, (b, r) in enumerate(zip(blobs, refs)):
        want, size, bs, posts = O.create(b, 2 << 20, salt=blob_salt)
        assert r.root.ref.marshal_binary() == want, (i, len(b))
        assert (r.root.size, r.root.block_size, r.type) == (len(b), 2 << 20, "blob")
        assert store.log[i][:2] == (posts[0][0], posts[0][1])
        assert store.blobs[want[:32]] == posts[0][3]


def test_post_blobs_device_config4_sample(gpu, O):
    """Config 4 shape on device: 65536 x 4 KiB distinct blobs (splitmix seed =
    blob index region); sampled roots vs the oracle."""
    torch = _torch()
    from glfs_amd import _native as N
    n, ln = 65536, 4096
    t = dev_bytes(torch, n * ln, seed=4)
    offs = torch.arange(n, dtype=torch.int64, device="cuda") * ln
    lens = torch.full((n,), ln, dtype=torch.int64, device="cuda")
    roots = zeros(torch, 64 * n)
    ct = zeros(torch, n * ln)
    blob_salt = O.derive_key(bytes(32), b"blob")
    N.check(N.lib.glfsx_post_blobs_device(2 << 20, blob_salt, None, t.data_ptr(),
                                          offs.data_ptr(), lens.data_ptr(), n, ln,
                                          ct.data_ptr(), roots.data_ptr(), None))
    torch.cuda.synchronize()
    rh = host(roots, 64 * n)
    data = host(t, n * ln)
    rng = random.Random(5)
    for i in [0, 1, n - 1] + rng.sample(range(n), 20):
        want = O.create(data[i * ln:(i + 1) * ln], 2 << 20, salt=blob_salt)[0]
        assert rh[64 * i:64 * i + 64] == want, i


@pytest.mark.parametrize("bulk", [False, True])
@pytest.mark.parametrize("ln", [1024, 2048, 4096, 8192, 16384])
def test_post_blobs_dense_vs_scattered(gpu, O, latency_wgs, ln, bulk):
    """Densely packed equal blobs take the LDS-staged wave path of k_small;
    the same blobs at permuted offsets take the per-lane path.  Every root
    and every ctext byte must agree (and sampled roots with the oracle), with
    and without ctext, with a partial last wave; latency-mode launches (the
    compiler's ARX form) and bulk ones (latency threshold 0: k_small_q,
    whose last blobs go as fine items of G lanes per blob, G = 2/4/8/16)."""
    torch = _torch()
    from glfs_amd import _native as N
    if bulk:
        latency_wgs(0)
    n = 64 * 5 + 17
    rng = random.Random(ln)
    perm = list(range(n))
    rng.shuffle(perm)
    blob_salt = O.derive_key(bytes(32), b"blob")
    a = dev_bytes(torch, n * ln, seed=ln)
    pi = torch.tensor(perm, dtype=torch.int64, device="cuda")
    b = torch.empty_like(a)
    b[:n * ln].view(n, ln)[pi] = a[:n * ln].view(n, ln)
    torch.cuda.synchronize()
    lens = torch.full((n,), ln, dtype=torch.int64, device="cuda")

    def run(src, offs, with_ct):
        roots = zeros(torch, 64 * n)
        ct = zeros(torch, n * ln) if with_ct else None
        N.check(N.lib.glfsx_post_blobs_device(2 << 20, blob_salt, None, src.data_ptr(),
                                              offs.data_ptr(), lens.data_ptr(), n, ln,
                                              ct.data_ptr() if with_ct else None,
                                              roots.data_ptr(), None))
        torch.cuda.synchronize()
        return host(roots, 64 * n), (host(ct, n * ln) if with_ct else None)

    dense = torch.arange(n, dtype=torch.int64, device="cuda") * ln
    ra, ca = run(a, dense, True)
    rb, cb = run(b, pi * ln, True)
    assert ra == rb
    assert all(ca[i * ln:(i + 1) * ln] == cb[perm[i] * ln:(perm[i] + 1) * ln]
               for i in range(n))
    assert run(a, dense, False)[0] == ra
    data = host(a, n * ln)
    for i in [0, 63, 64, n - 1] + rng.sample(range(n), 4):
        want, _, _, posts = O.create(data[i * ln:(i + 1) * ln], 2 << 20, salt=blob_salt)
        assert ra[64 * i:64 * i + 64] == want, i
        assert ca[i * ln:(i + 1) * ln] == posts[0][3], i


def test_post_blobs_bulk_mixed_vs_oracle(gpu, O, latency_wgs):
    """k_small in a bulk launch (the asm ARX form) over blobs of at most 4 KiB:
    waves of densely packed 4 KiB blobs (LDS-staged), waves mixing them with
    ragged, empty and unaligned blobs (per-lane paths), and a partial last
    wave; every root and ctext byte against the oracle."""
    torch = _torch()
    from glfs_amd import _native as N
    latency_wgs(0)
    rng = random.Random(23)
    lens = [4096] * 320 + [0, 1, 63, 64, 1024, 2049, 4095, 4096, 4096, 3000]
    lens += [rng.choice([4096, rng.randrange(0, 4097)]) for _ in range(300)] + [4096] * 77
    offs, o = [], 0
    for i, n in enumerate(lens):
        if i >= 320 and rng.random() < 0.3:
            o += rng.randrange(1, 16)          # unaligned / scattered blobs
        offs.append(o)
        o += n
    total = o
    src = dev_bytes(torch, total + 64, seed=29)
    ct = zeros(torch, total + 64)
    roots = zeros(torch, 64 * len(lens))
    d_offs = torch.tensor(offs, dtype=torch.int64, device="cuda")
    d_lens = torch.tensor(lens, dtype=torch.int64, device="cuda")
    blob_salt = O.derive_key(bytes(32), b"blob")
    N.check(N.lib.glfsx_post_blobs_device(2 << 20, blob_salt, None, src.data_ptr(),
                                          d_offs.data_ptr(), d_lens.data_ptr(), len(lens),
                                          max(lens), ct.data_ptr(), roots.data_ptr(), None))
    torch.cuda.synchronize()
    data, ch, rh = host(src, total), host(ct, total), host(roots, 64 * len(lens))
    for i, (o, n) in enumerate(zip(offs, lens)):
        want, _, _, posts = O.create(data[o:o + n], 2 << 20, salt=blob_salt)
        assert rh[64 * i:64 * i + 64] == want, (i, n)
        assert ch[o:o + n] == posts[0][3], (i, n)


# ---------------------------------------------------------------- read side
@pytest.mark.parametrize("bs,size", [(1 << 20, (9 << 20) + 77), (4096, 4096 * 33 + 5),
                                     (128, 128 * 7), (8192, 8192 * 3 + 100),
                                     (8192, 8192 * 5), (65536, 65536 * 2 + 8191),
                                     (2 << 20, (2 << 20) + 8192 + 64)])
def test_decrypt_batch_roundtrip(gpu, O, bs, size):
    """getF (ref.go:113-126): decrypting every posted data block with its DEK
    gives back the plaintext; block 0 also checked against the oracle."""
    torch = _torch()
    from glfs_amd import _native as N
    raw = O.derive_key(bytes(32), b"raw")
    n = -(-size // bs)
    t = dev_bytes(torch, size, seed=31)
    ct = zeros(torch, size + 64)
    refs = zeros(torch, 64 * n)
    pt = zeros(torch, size + 64)
    N.check(N.lib.glfsx_post_batch_device(raw, t.data_ptr(), size, bs, ct.data_ptr(),
                                          refs.data_ptr(), None, None))
    N.check(N.lib.glfsx_decrypt_batch_device(ct.data_ptr(), size, bs, refs.data_ptr(),
                                             pt.data_ptr(), None))
    torch.cuda.synchronize()
    assert torch.equal(pt[:size], t[:size])
    assert not pt[size:].any()   # nothing written past the end
    r0 = host(refs, 64)
    assert O.chacha20_xor(host(ct, min(bs, size)), r0[32:]) == host(t, min(bs, size))
    # unaligned destination: the bulk line kernel is bypassed, same bytes
    pt2 = zeros(torch, size + 64)
    N.check(N.lib.glfsx_decrypt_batch_device(ct.data_ptr(), size, bs, refs.data_ptr(),
                                             pt2.data_ptr() + 1, None))
    torch.cuda.synchronize()
    assert torch.equal(pt2[1:size + 1], t[:size])


# ------------------------------------------------- writer pipeline, extremes
def test_writer_pipeline_many_batches(gpu, O):
    """bs 4 KiB (bf 64): a 64 MiB batch holds 16384 blocks, so ~3 batches go
    through the three-slot pipeline while index nodes are posted mid-batch;
    the full Post sequence must equal the reference writer's."""
    from glfs_amd import bigblob
    bs = 4096
    size = 3 * (64 << 20) + 12345
    data = O.fill_splitmix(size, 77)
    want_root, _, _, want_posts = O.create(data, bs, salt=None, chunks=[size // 3, size])
    store = bigblob.MemStore(bs)
    w = bigblob.Machine(bs).new_writer(store)
    w.write(data[:size // 3])
    w.write(data[size // 3:])
    root = w.finish()
    w.close()
    assert root.ref.marshal_binary() == want_root
    assert len(store.log) == len(want_posts)
    assert [r for _, r, _ in store.log] == [r for _, r, _, _ in want_posts]


def test_huge_block_size_g64(gpu, O):
    """16 MiB blocks use the G = 64 kernels (64 chunks per lane)."""
    from glfs_amd import bigblob
    bs = 16 << 20
    data = O.fill_splitmix(bs + 777, 8)
    refs, ct = _post_batch_host(bytes(32), data, bs)
    for j in range(2):
        r, c = O.post(bytes(32), data[j * bs:(j + 1) * bs])
        assert refs[64 * j:64 * j + 64] == r
    assert bigblob.derive_key(bytes(32), data[:bs]) == O.derive_key(bytes(32), data[:bs])


def test_writer_keyed_cid_and_tiny_writes(gpu, O):
    """A store whose CID is keyed (cid_key), fed one byte at a time."""
    from glfs_amd import bigblob
    key = bytes(range(7, 39))
    data = O.fill_splitmix(3000, 9)
    want_root, _, _, want_posts = O.create(data, 1024, salt=None, cid_key=key)
    store = bigblob.MemStore(1024)
    w = bigblob.Machine(1024).new_writer(store, None, cid_key=key)
    for i in range(len(data)):
        w.write(data[i:i + 1])
    root = w.finish()
    w.close()
    assert root.ref.marshal_binary() == want_root
    assert [r for _, r, _ in store.log] == [r for _, r, _, _ in want_posts]


def test_concat_vs_oracle(gpu, O):
    """blob.go:333-345 Concat: the roots' bytes, read back through the GPU
    decrypt, re-written as one blob == the oracle's Create of the joined
    bytes; block_size is ignored as in the reference."""
    from glfs_amd import bigblob
    bs = 1024
    store = bigblob.MemStore(bs)
    m = bigblob.Machine(bs)
    parts = [O.fill_splitmix(n, 50 + n) for n in (0, 5000, 1024, 16 * 1024 + 3)]
    roots = [m.create(store, None, p) for p in parts]
    got = m.concat(store, 12345, None, *roots)
    want = O.create(b"".join(parts), bs, salt=None)[0]
    assert got.ref.marshal_binary() == want
    assert got.size == sum(map(len, parts))


def test_post_blobs_mixed_sizes(gpu, O):
    """glfs.PostBlob batched over blobs of every size class: <= 16 KiB (one
    lane each), one block above 16 KiB, exactly one block, and several
    blocks (a whole Create with an index node): every root and the whole
    Post sequence equal n sequential reference PostBlob calls."""
    import torch
    from glfs_amd import _native as N, bigblob, glfs
    bs = 2 << 20
    lens = [0, 5, 16384, 16385, 100_000, bs - 1, bs, bs + 1, 3 * bs + 5, 4096, 0, 77]
    blobs = [O.fill_splitmix(n, 300 + i) for i, n in enumerate(lens)]
    blob_salt = O.derive_key(bytes(32), b"blob")
    store = bigblob.MemStore(bs)
    refs = glfs.Machine().post_blobs(store, blobs)
    want_log = []
    for i, b in enumerate(blobs):
        want, size, _, posts = O.create(b, bs, salt=blob_salt)
        assert refs[i].root.ref.marshal_binary() == want, (i, len(b))
        assert refs[i].root.size == len(b)
        want_log += [(k, r) for k, r, _, _ in posts]
        for _, r, _, c in posts:             # every ctext the store got
            assert store.blobs[r[:32]] == c, (i, len(b))
    assert [(k, r) for k, r, _ in store.log] == want_log
    # device-resident: the same roots, ctext of every blob in place
    offs, pos = [], 0
    for b in blobs:
        offs.append(pos)
        pos += len(b) + 13          # unaligned, gaps between blobs
    d = torch.zeros(pos + 64, dtype=torch.uint8, device="cuda")
    for o, b in zip(offs, blobs):
        if b:
            d[o:o + len(b)] = torch.tensor(list(b), dtype=torch.uint8, device="cuda") \
                if len(b) < 100_000 else torch.frombuffer(bytearray(b), dtype=torch.uint8).cuda()
    roots = torch.zeros(64 * len(blobs), dtype=torch.uint8, device="cuda")
    ct = torch.zeros_like(d)
    do = torch.tensor(offs, dtype=torch.int64, device="cuda")
    dl = torch.tensor(lens, dtype=torch.int64, device="cuda")
    N.check(N.lib.glfsx_post_blobs_device(bs, blob_salt, None, d.data_ptr(), do.data_ptr(),
                                          dl.data_ptr(), len(blobs), max(lens), ct.data_ptr(),
                                          roots.data_ptr(), None))
    torch.cuda.synchronize()
    rh = bytes(roots.cpu().numpy().tobytes())
    cth = bytes(ct.cpu().numpy().tobytes())
    for i, b in enumerate(blobs):
        assert rh[64 * i:64 * i + 64] == refs[i].root.ref.marshal_binary(), i
        if 0 < len(b) <= bs:
            assert cth[offs[i]:offs[i] + len(b)] == O.post(O.derive_key(blob_salt, b"raw"), b)[1]


def test_derive_key_xof_any_length(gpu, O):
    """ref.go:152-161 with len(out) > 32 (the XOF beyond the digest: output
    blocks 0, 1, ... of the root node) and with inputs that take the
    streaming hasher: every byte vs the oracle's XOF, which
    tests/test_oracle.py pins against upstream BLAKE3 C."""
    from glfs_amd import bigblob
    rng = random.Random(9)
    salt = bytes(rng.randrange(256) for _ in range(32))
    for n in [0, 1, 63, 64, 65, 1023, 1024, 1025, 2048, 5000, 256 * 1024 - 1, 256 * 1024,
              256 * 1024 + 1, 3 * 256 * 1024 + 4097, 1 << 22]:
        data = O.fill_splitmix(n, n + 3)
        for out_len in (33, 64, 65, 131, 1000):
            assert bigblob.derive_key(salt, data, out_len) == O.blake3(data, salt, out_len), \
                (n, out_len)
        # the first 32 bytes equal the digest path's
        assert bigblob.derive_key(salt, data, 40)[:32] == bigblob.derive_key(salt, data), n


def test_derive_key_input_above_4gib(gpu, O):
    """An input longer than the write path's 4 GiB message limit: 4 GiB +
    1 MiB + 5 bytes through the streaming hasher (17 slabs), 32 and 100 bytes
    of output vs the oracle (threaded over the chunks is not available for a
    single keyed message, so the reference is upstream BLAKE3 C when the
    image has it, else the oracle)."""
    import refimpl as R
    from glfs_amd import bigblob
    n = (4 << 30) + (1 << 20) + 5
    data = O.fill_splitmix(n, 77)
    salt = bytes(range(32))
    want = (R.blake3(data, salt, 100) if R.blake3_lib() is not None
            else O.blake3(data, salt, 100))
    assert bigblob.derive_key(salt, data, 100) == want
    assert bigblob.derive_key(salt, data, 32) == want[:32]

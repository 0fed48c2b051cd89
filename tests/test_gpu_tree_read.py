"""GPU parity for the paths either side of the write path:
trees (tree.go PostTree/TreeWriter -> the tree JSON bytes through the GPU
Writer), the read side (ReadAt/getPiece/getF/Reader over the GPU ChaCha20),
and Sync/Populate/Traverse.  The tree blob's root is compared with the
oracle's Create of the same bytes under typeSalt("tree"); the line bytes are
pinned by tests/test_tree_host.py (except the cid field: parity unpinned)."""
import random

import pytest

pytestmark = pytest.mark.gpu

KIB, MIB = 1 << 10, 1 << 20


def _tree_salt(O):
    return O.derive_key(bytes(32), b"tree")


def _oracle_tree_root(O, ents):
    from glfs_amd import tree as T
    data = b"".join(T.entry_json_line(e) for e in ents)
    return O.create(data, 2 * MIB, salt=_tree_salt(O), store_max=2 * MIB)[0], len(data)


def test_post_tree_map_vs_oracle(gpu, O):
    from glfs_amd import bigblob, glfs, tree as T
    s = bigblob.MemStore(2 * MIB)
    m = glfs.Machine()
    files = {"b.txt": b"hello", "a.txt": b"", "c<&>.bin": O.fill_splitmix(5000, 3)}
    refs = {k: m.post_blob(s, v) for k, v in files.items()}
    tref = m.post_tree_map(s, refs)
    assert tref.type == "tree"
    ents = sorted((T.TreeEntry(k, 0o644, v) for k, v in refs.items()),
                  key=lambda e: e.name.encode())
    want, n = _oracle_tree_root(O, ents)
    assert tref.root.ref.marshal_binary() == want
    assert (tref.root.size, tref.root.block_size) == (n, 2 * MIB)
    # read back through the GPU decrypt
    got = m.get_tree_slice(s, tref)
    assert got == ents
    for e in got:
        assert m.get_blob_bytes(s, e.ref, 1 << 30) == files[e.name]
    with pytest.raises(glfs.ErrRefType):
        m.get_blob(s, tref)


def test_post_tree_nested_paths(gpu, O):
    """tree.go:195-238: entries with paths become subtrees posted first."""
    from glfs_amd import bigblob, glfs, tree as T
    s = bigblob.MemStore(2 * MIB)
    m = glfs.Machine()
    paths = ["e.txt", "a/d.txt", "a/b/c.txt", "/a/b/z.txt/", "q/r/s/t"]
    refs = {p: m.post_blob(s, p.encode() * 3) for p in paths}
    root = m.post_tree(s, [T.TreeEntry(p, 0o644, r) for p, r in refs.items()])

    def walk(ref, prefix=""):
        out = {}
        ents = m.get_tree_slice(s, ref)
        # each tree blob equals the oracle's Create of its own line bytes
        assert ref.root.ref.marshal_binary() == _oracle_tree_root(O, ents)[0]
        for e in ents:
            p = (prefix + "/" + e.name) if prefix else e.name
            if e.ref.type == "tree":
                assert e.file_mode == T.MODE_TREE
                out.update(walk(e.ref, p))
            else:
                out[p] = e.ref
        return out

    flat = walk(root)
    assert flat == {T.clean_path(p): r for p, r in refs.items()}
    # a lone entry with an empty cleaned path is returned as-is
    one = m.post_blob(s, b"x")
    assert m.post_tree(s, [T.TreeEntry("/", 0o644, one)]) == one


def test_tree_writer_errors(gpu):
    from glfs_amd import bigblob, glfs, tree as T
    s = bigblob.MemStore(2 * MIB)
    m = glfs.Machine()
    r = m.post_blob(s, b"data")
    tw = m.new_tree_writer(s)
    tw.put(T.TreeEntry("b", 0o644, r))
    with pytest.raises(T.TreeError, match="out of order"):
        tw.put(T.TreeEntry("a", 0o644, r))
    with pytest.raises(T.TreeError, match="out of order"):
        tw.put(T.TreeEntry("b", 0o644, r))
    ghost = glfs.Ref("blob", bigblob.Root(bigblob.Ref(b"\x01" * 32, b"\x02" * 32), 1, 2 * MIB))
    with pytest.raises(T.TreeError, match="referential integrity"):
        tw.put(T.TreeEntry("c", 0o644, ghost))
    tw.put(T.TreeEntry("d", 0o644, r))
    ref = tw.finish()
    assert [e.name for e in m.get_tree_slice(s, ref)] == ["b", "d"]


class _TrustingStore:
    """Store whose Exists is always true: exercises multi-chunk trees over
    synthetic refs (the tree writer does not read the entries' blobs)."""

    def __init__(self):
        self.inner = 0
        from glfs_amd import bigblob
        self.s = bigblob.MemStore(2 * MIB)

    def max_size(self):
        return self.s.max_size()

    def post(self, ct, ref, kind=0):
        self.s.post(ct, ref, kind)

    def exists(self, cid):
        return True

    def get(self, cid):
        return self.s.get(cid)


def test_config4_tree_multi_chunk(gpu, O):
    """Config 4's directory shape ("%07d" names, 4 KiB blobs) at 12k entries:
    ~3 MiB of JSON = 2 data chunks + 1 index node of the tree blob."""
    from glfs_amd import bigblob, glfs, tree as T
    st = _TrustingStore()
    m = glfs.Machine()
    rng = random.Random(4)
    ents = []
    for i in range(12_000):
        root = bigblob.Root(bigblob.Ref(rng.randbytes(32), rng.randbytes(32)), 4096, 2 * MIB)
        ents.append(T.TreeEntry("%07d" % i, 0o644, glfs.Ref("blob", root)))
    tref = m.post_tree_slice(st, ents)
    want, n = _oracle_tree_root(O, ents)
    assert n > 2 * MIB
    assert tref.root.ref.marshal_binary() == want and tref.root.size == n
    assert [k for k, _, _ in st.s.log] == [0, 0, 1]
    assert m.get_tree_slice(st, tref) == ents


def test_config4_end_to_end_sample(gpu, O):
    """Config 4 end to end on a 2048-blob sample: batched PostBlob (one lane
    per blob) -> PostTreeMap -> tree root vs the oracle."""
    from glfs_amd import bigblob, glfs, tree as T
    s = bigblob.MemStore(2 * MIB)
    m = glfs.Machine()
    n = 2048
    blobs = [O.fill_splitmix(4096, i) for i in range(n)]
    refs = m.post_blobs(s, blobs)
    blob_salt = O.derive_key(bytes(32), b"blob")
    for i in (0, 1, n // 2, n - 1):
        assert refs[i].root.ref.marshal_binary() == O.create(
            blobs[i], 2 * MIB, salt=blob_salt, store_max=2 * MIB)[0]
    tref = m.post_tree_map(s, {"%07d" % i: r for i, r in enumerate(refs)})
    ents = [T.TreeEntry("%07d" % i, 0o644, r) for i, r in enumerate(refs)]
    assert tref.root.ref.marshal_binary() == _oracle_tree_root(O, ents)[0]


# ----------------------------------------------------------------- read side
def test_read_at_semantics(gpu, O):
    """blob.go:31-51: ReadAt returns bytes from ONE block only, and io.EOF
    exactly when the read ends at Size."""
    from glfs_amd import bigblob
    bs = 1024
    s = bigblob.MemStore(bs)
    m = bigblob.Machine(bs)
    data = O.fill_splitmix(16 * 16 * bs + 777, 9)  # depth 3
    root = m.create(s, None, data)
    assert bigblob.depth(root.size, bs) == 3
    rng = random.Random(5)
    for _ in range(60):
        off = rng.randrange(len(data))
        want_n = rng.randrange(1, 3 * bs)
        got, eof = m.read_at(s, root, off, want_n)
        blk_end = min((off // bs + 1) * bs, len(data))
        assert got == data[off:min(off + want_n, blk_end)]
        assert eof == (off + len(got) == len(data))
    got, eof = m.read_at(s, root, len(data) - 5, 100)
    assert got == data[-5:] and eof
    r = m.new_reader(s, root)
    assert r.read() == data
    assert r.read(10) == b""
    r.seek(-100, r.SEEK_END)
    assert r.read(1000) == data[-100:]
    r.seek(5)
    r.seek(10, r.SEEK_CUR)
    assert r.read(20) == data[15:35]
    assert r.read_at(30, 2 * bs - 10)[0] == data[2 * bs - 10:2 * bs]


def test_get_f_cache_lru(gpu, O):
    from glfs_amd import bigblob
    bs = 1024
    s = bigblob.MemStore(bs)
    m = bigblob.Machine(bs, cache_size=4)
    root = m.create(s, None, O.fill_splitmix(20 * bs, 2))
    assert m.new_reader(s, root).read() == O.fill_splitmix(20 * bs, 2)
    assert len(m._cache) == 4


def test_sync_and_populate(gpu, O):
    """blob.go:270-331: Sync copies every reachable blob (children first) and
    is a no-op when dst has the root; Populate adds every reachable CID."""
    from glfs_amd import bigblob
    bs = 1024
    src = bigblob.MemStore(bs)
    m = bigblob.Machine(bs)
    data = O.fill_splitmix(16 * bs * 3 + 100, 6)  # depth 2: 49 data + 4 + 1 index
    root = m.create(src, None, data)
    dst = bigblob.MemStore(bs)
    seen = []
    m.sync(dst, src, root, lambda r: seen.append(r.read(10)))
    assert seen == [data[:10]]
    assert set(dst.blobs) == set(src.blobs)
    assert dst.log[-1][1][:32] == root.ref.cid  # the root is copied last
    assert m.new_reader(dst, root).read() == data
    n_posts = len(dst.log)
    m.sync(dst, src, root)  # dst has the root: nothing happens
    assert len(dst.log) == n_posts
    cids = bigblob.CIDSet()
    m.populate(src, root, cids)
    assert cids.cids == set(src.blobs)
    order = []
    m.traverse(src, root, lambda cid: True, lambda lvl, ref: order.append(lvl))
    assert order[-1] == bigblob.depth(root.size, bs) and order.count(0) == 49


# ------------------------------------------------------ config 4, full size
def _dev_arr(torch, vals, dtype):
    return torch.tensor(vals, dtype=dtype, device="cuda")


def _encode_device(torch, ents, out_shift=0, cap=None, want_ends=True, roots_shift=0):
    """glfsx_tree_encode_device over entries copied to HBM (the roots array
    roots_shift bytes past a 16-B boundary); returns (bytes, line_ends) or
    raises GlfsxError."""
    import ctypes
    from glfs_amd import _native as N, tree as T
    n = len(ents)
    names = [T.go_bytes(e.name) for e in ents]
    types = [T.go_bytes(e.ref.type) for e in ents]

    def offs(parts):
        o, acc = [0], 0
        for p in parts:
            acc += len(p)
            o.append(acc)
        return o

    u8 = lambda b: torch.tensor(list(b) or [0], dtype=torch.uint8, device="cuda")
    d_names, d_types = u8(b"".join(names)), u8(b"".join(types))
    d_no, d_to = _dev_arr(torch, offs(names), torch.int64), _dev_arr(torch, offs(types), torch.int64)
    d_modes = _dev_arr(torch, [e.file_mode for e in ents], torch.int64).to(torch.int32)
    d_roots = u8(bytes(roots_shift) + b"".join(e.ref.root.ref.cid + e.ref.root.ref.dek
                                              for e in ents))[roots_shift:]
    d_sizes = _dev_arr(torch, [e.ref.root.size for e in ents], torch.int64)
    d_bss = _dev_arr(torch, [e.ref.root.block_size for e in ents], torch.int64)
    total = ctypes.c_uint64()
    N.check(N.lib.glfsx_tree_encode_device(n, d_names.data_ptr(), d_no.data_ptr(),
                                           d_modes.data_ptr(), d_types.data_ptr(),
                                           d_to.data_ptr(), d_roots.data_ptr(),
                                           d_sizes.data_ptr(), d_bss.data_ptr(), None, 0,
                                           None, ctypes.byref(total), None))
    ln = total.value
    out = torch.full((ln + 64,), 0xA5, dtype=torch.uint8, device="cuda")
    ends = torch.zeros(n, dtype=torch.int64, device="cuda")
    rc = N.lib.glfsx_tree_encode_device(n, d_names.data_ptr(), d_no.data_ptr(),
                                        d_modes.data_ptr(), d_types.data_ptr(),
                                        d_to.data_ptr(), d_roots.data_ptr(),
                                        d_sizes.data_ptr(), d_bss.data_ptr(),
                                        out.data_ptr() + out_shift,
                                        ln if cap is None else cap,
                                        ends.data_ptr() if want_ends else None,
                                        ctypes.byref(total), None)
    torch.cuda.synchronize()
    o = bytes(out.cpu().numpy().tobytes())
    if rc:
        assert set(o) == {0xA5}, "nothing may be written on error"
        N.check(rc)
    assert set(o[:out_shift]) <= {0xA5} and set(o[out_shift + ln:]) <= {0xA5}
    return o[out_shift:out_shift + ln], ends.cpu().tolist()


def test_tree_encode_device_vs_host(gpu):
    """k_tree_len/prefix/write == the host encoder == entry_json_line, for
    every escaping class, several destination and roots alignments, lines too long
    for a workgroup's LDS image, and a too-small buffer (an error, nothing
    written)."""
    import torch
    from glfs_amd import _native as N, bigblob, glfs, tree as T
    rng = random.Random(17)
    pool = ["plain", "<a&b>", "\n\r\t\b\f\x00\x1f\x7f", "é日本\U0001F600", "bad\udc80\udcff",
            "q\"b\\s", " x ", "%07d" % 5, "\udced\udca0\udc80"]
    ents = []
    for i in range(3000):
        name = rng.choice(pool) + str(i) + rng.choice(pool)
        if i % 700 == 3:
            name = "L" * rng.randrange(300, 2000) + name   # forces the byte path
        r = glfs.Ref(rng.choice(["blob", "tree", "<&>"]),
                     bigblob.Root(bigblob.Ref(rng.randbytes(32), rng.randbytes(32)),
                                  rng.randrange(1 << 63), rng.choice([128, 2 << 20])))
        ents.append(T.TreeEntry(name, rng.choice([0o644, T.MODE_TREE]), r))
    want, want_ends = T.encode_lines(ents)
    assert want == b"".join(T.entry_json_line(e) for e in ents)
    for shift in (0, 1, 7, 15):
        got, ends = _encode_device(torch, ents, out_shift=shift)
        assert got == want, shift
        assert ends == want_ends
    for rs in (1, 4, 8):   # refs read bytewise when not 16-B aligned
        assert _encode_device(torch, ents, out_shift=3, roots_shift=rs)[0] == want, rs
    with pytest.raises(N.GlfsxError):
        _encode_device(torch, ents, cap=len(want) - 1)


def test_fill_blobs_matches_oracle(gpu, O):
    import ctypes
    import torch
    from glfs_amd import _native as N
    n, ln = 1000, 4096
    t = torch.empty(n * ln, dtype=torch.uint8, device="cuda")
    N.check(N.lib.glfsx_fill_splitmix_blobs_device(t.data_ptr(), n, ln, 17, None))
    torch.cuda.synchronize()
    want = ctypes.create_string_buffer(n * ln)
    O.lib().oracle_fill_splitmix_blobs(want, n, ln, 17)
    assert bytes(t.cpu().numpy().tobytes()) == want.raw
    assert want.raw[5 * ln:6 * ln] == O.fill_splitmix(ln, 22)


def test_config4_full_size_end_to_end(gpu, O):
    """BASELINE config 4 at its stated size: 1,048,576 distinct 4 KiB blobs
    (blob i = splitmix stream of seed i) -> glfs.Machine.post_blobs (the
    store receives every Post in order) -> PostTreeMap with "%07d" names.
    Every one of the 1M roots vs the threaded oracle; the tree root vs the
    oracle's Create of the tree bytes (encoded by entry_json_line, an
    independent encoder) under typeSalt("tree").  Then the device-resident
    route (post_blobs_device -> tree_encode_device -> create_device) must
    give the same tree root."""
    import ctypes
    import numpy as np
    import torch
    from glfs_amd import _native as N, bigblob, glfs, tree as T
    n, ln, bs = 1 << 20, 4096, 2 * MIB
    d = torch.empty(n * ln, dtype=torch.uint8, device="cuda")
    N.check(N.lib.glfsx_fill_splitmix_blobs_device(d.data_ptr(), n, ln, 0, None))
    torch.cuda.synchronize()
    host = d.cpu().numpy()
    hb = host.tobytes()
    blobs = [hb[i * ln:(i + 1) * ln] for i in range(n)]
    # ------------------------------------------------ the Python API route
    s = bigblob.MemStore(bs)
    m = glfs.Machine()
    refs = m.post_blobs(s, blobs)
    print("config4: posted", n, "blobs", flush=True)
    assert len(s.log) == n
    blob_salt = O.derive_key(bytes(32), b"blob")
    raw = O.derive_key(blob_salt, b"raw")
    want = np.empty(64 * n, dtype=np.uint8)
    O.lib().oracle_post_batch(want.ctypes.data, None, raw, host.ctypes.data, n * ln, ln,
                              None, 16)
    want_b = want.tobytes()
    got_b = b"".join(r.root.ref.marshal_binary() for r in refs)
    assert got_b == want_b                       # every root, bit-exact
    assert all(r.root.size == ln and r.root.block_size == bs for r in refs)
    assert [k for k, _, _ in s.log[:3]] == [0, 0, 0]
    assert s.log[n - 1][1] == want_b[64 * (n - 1):]
    del blobs
    tref = m.post_tree_map(s, {"%07d" % i: r for i, r in enumerate(refs)})
    print("config4: tree posted", flush=True)
    ents = [T.TreeEntry("%07d" % i, 0o644, r) for i, r in enumerate(refs)]
    tree_bytes = b"".join(T.entry_json_line(e) for e in ents)
    tsalt = O.derive_key(bytes(32), b"tree")
    want_root, size, _, want_posts = O.create(tree_bytes, bs, salt=tsalt, store_max=bs)
    assert tref.root.ref.marshal_binary() == want_root
    assert tref.root.size == size == len(tree_bytes)
    assert [r for _, r, _ in s.log[n:]] == [r for _, r, _, _ in want_posts]
    # --------------------------------------------- the device-resident route
    roots = torch.empty(64 * n, dtype=torch.uint8, device="cuda")
    offs = torch.arange(n, dtype=torch.int64, device="cuda") * ln
    lens = torch.full((n,), ln, dtype=torch.int64, device="cuda")
    N.check(N.lib.glfsx_post_blobs_device(bs, blob_salt, None, d.data_ptr(), offs.data_ptr(),
                                          lens.data_ptr(), n, ln, None, roots.data_ptr(), None))
    names = torch.tensor(np.frombuffer("".join("%07d" % i for i in range(n)).encode(),
                                       dtype=np.uint8), device="cuda")
    name_offs = torch.arange(n + 1, dtype=torch.int64, device="cuda") * 7
    types = torch.tensor(np.frombuffer(b"blob" * n, dtype=np.uint8), device="cuda")
    type_offs = torch.arange(n + 1, dtype=torch.int64, device="cuda") * 4
    modes = torch.full((n,), 0o644, dtype=torch.int32, device="cuda")
    bss = torch.full((n,), bs, dtype=torch.int64, device="cuda")
    out = torch.empty(len(tree_bytes) + 64, dtype=torch.uint8, device="cuda")
    total = ctypes.c_uint64()
    N.check(N.lib.glfsx_tree_encode_device(n, names.data_ptr(), name_offs.data_ptr(),
                                           modes.data_ptr(), types.data_ptr(),
                                           type_offs.data_ptr(), roots.data_ptr(),
                                           lens.data_ptr(), bss.data_ptr(), out.data_ptr(),
                                           out.numel(), None, ctypes.byref(total), None))
    assert total.value == len(tree_bytes)
    assert bytes(out[:total.value].cpu().numpy().tobytes()) == tree_bytes
    r = N.glfsx_root()
    N.check(N.lib.glfsx_create_device(bs, tsalt, None, out.data_ptr(), total.value, None,
                                      ctypes.byref(r), None, None))
    assert bytes(r.ref) == want_root
    # ------------------------------- the same in one pipelined call
    roots2 = torch.zeros(64 * n, dtype=torch.uint8, device="cuda")
    out2 = torch.zeros(len(tree_bytes) + 64, dtype=torch.uint8, device="cuda")
    r2, total2 = N.glfsx_root(), ctypes.c_uint64()
    N.check(N.lib.glfsx_post_tree_device(n, bs, blob_salt, tsalt, None, d.data_ptr(),
                                         offs.data_ptr(), lens.data_ptr(), ln, None,
                                         roots2.data_ptr(), names.data_ptr(),
                                         name_offs.data_ptr(), modes.data_ptr(),
                                         types.data_ptr(), type_offs.data_ptr(), bss.data_ptr(),
                                         bs, out2.data_ptr(), out2.numel(), None,
                                         ctypes.byref(r2), ctypes.byref(total2), None))
    torch.cuda.synchronize()
    assert bytes(r2.ref) == want_root and r2.size == len(tree_bytes)
    assert total2.value == len(tree_bytes)
    assert bytes(roots2.cpu().numpy().tobytes()) == want_b
    assert bytes(out2[:total2.value].cpu().numpy().tobytes()) == tree_bytes


def _tree_inputs(torch, names, types, modes, sizes, bss):
    import numpy as np
    nb = b"".join(names)
    tb = b"".join(types)
    no = np.cumsum([0] + [len(x) for x in names]).astype(np.int64)
    to = np.cumsum([0] + [len(x) for x in types]).astype(np.int64)
    cuda = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
    return (cuda(np.frombuffer(nb or b"\0", dtype=np.uint8)), cuda(no),
            cuda(np.array(modes, dtype=np.int32)), cuda(np.frombuffer(tb or b"\0", dtype=np.uint8)),
            cuda(to), cuda(np.array(sizes, dtype=np.int64)), cuda(np.array(bss, dtype=np.int64)))


@pytest.mark.parametrize("n,tree_bs", [(70_000, 2 * MIB), (3000, 4096), (300, 64 * 1024),
                                       (1, 2 * MIB), (257, 1024),
                                       # one tree block at 8 MiB (its ref is
                                       # the root); 5 blocks + an index node
                                       (20_000, 8 * MIB), (20_000, MIB),
                                       # 3 blocks; 2 x 64 KiB per block, the
                                       # last one partial
                                       (40_000, 4 * MIB), (2_500, 128 * 1024)])
def test_post_tree_device_equals_sequence(gpu, O, n, tree_bs):
    """glfsx_post_tree_device (blob hashing and tree lines overlapped; the
    tree blob's blocks posted by the general post, launch_post) against the
    three calls in
    sequence on the same inputs: ragged blob sizes 0..16 KiB at odd offsets,
    names with JSON escapes and non-ASCII bytes, every blob root, every
    line byte, the tree root."""
    import ctypes
    import random
    import torch
    from glfs_amd import _native as N
    rng = random.Random(n * 7 + tree_bs)
    lens_h = [rng.choice([0, 1, 63, 100, 1024, 4096, 5000, 16384, rng.randrange(16385)])
              for _ in range(n)]
    offs_h, o = [], 0
    for ln in lens_h:
        offs_h.append(o)
        o += ln + rng.randrange(3)
    data = torch.empty(o + 64, dtype=torch.uint8, device="cuda")
    N.check(N.lib.glfsx_fill_splitmix_device(data.data_ptr(), 0, o + 8 - o % 8, n, None))
    names = [(b"n%06d" % i) + rng.choice([b"", b"\"", b"<&>", "é".encode(), b"\xff"])
             for i in range(n)]
    types = [rng.choice([b"blob", b"tree"]) for _ in range(n)]
    modes = [rng.choice([0o644, 0o755, 0o40000]) for _ in range(n)]
    bss = [2 * MIB] * n
    offs = torch.tensor(offs_h, dtype=torch.int64, device="cuda")
    lens = torch.tensor(lens_h, dtype=torch.int64, device="cuda")
    dn, dno, dm, dt, dto, _, dbs = _tree_inputs(torch, names, types, modes, lens_h, bss)
    bsalt, tsalt = O.derive_key(bytes(32), b"blob"), O.derive_key(bytes(32), b"tree")
    cap = 300 * n + 4096
    torch.cuda.synchronize()
    # the sequence
    roots1 = torch.zeros(64 * n, dtype=torch.uint8, device="cuda")
    N.check(N.lib.glfsx_post_blobs_device(2 * MIB, bsalt, None, data.data_ptr(),
                                          offs.data_ptr(), lens.data_ptr(), n, 16384, None,
                                          roots1.data_ptr(), None))
    out1 = torch.zeros(cap, dtype=torch.uint8, device="cuda")
    t1 = ctypes.c_uint64()
    N.check(N.lib.glfsx_tree_encode_device(n, dn.data_ptr(), dno.data_ptr(), dm.data_ptr(),
                                           dt.data_ptr(), dto.data_ptr(), roots1.data_ptr(),
                                           lens.data_ptr(), dbs.data_ptr(), out1.data_ptr(),
                                           cap, None, ctypes.byref(t1), None))
    r1 = N.glfsx_root()
    N.check(N.lib.glfsx_create_device(tree_bs, tsalt, None, out1.data_ptr(), t1.value, None,
                                      ctypes.byref(r1), None, None))
    # one call
    roots2 = torch.zeros(64 * n, dtype=torch.uint8, device="cuda")
    out2 = torch.zeros(cap, dtype=torch.uint8, device="cuda")
    r2, t2 = N.glfsx_root(), ctypes.c_uint64()
    for _ in range(2):   # twice: level buffers and counters reused
        N.check(N.lib.glfsx_post_tree_device(n, 2 * MIB, bsalt, tsalt, None, data.data_ptr(),
                                             offs.data_ptr(), lens.data_ptr(), 16384, None,
                                             roots2.data_ptr(), dn.data_ptr(), dno.data_ptr(),
                                             dm.data_ptr(), dt.data_ptr(), dto.data_ptr(),
                                             dbs.data_ptr(), tree_bs, out2.data_ptr(), cap,
                                             None, ctypes.byref(r2), ctypes.byref(t2), None))
        torch.cuda.synchronize()
        assert t2.value == t1.value
        assert bytes(r2.ref) == bytes(r1.ref)
        assert torch.equal(roots1, roots2)
        assert torch.equal(out1[:t1.value], out2[:t2.value])
    # and against the oracle's Create of the lines for the tree root
    want, _, _, _ = O.create(bytes(out1[:t1.value].cpu().numpy().tobytes()), tree_bs,
                             salt=tsalt, closed_form=True)
    assert bytes(r2.ref) == want
    with pytest.raises(N.GlfsxError):   # lines above the buffer
        N.check(N.lib.glfsx_post_tree_device(n, 2 * MIB, bsalt, tsalt, None, data.data_ptr(),
                                             offs.data_ptr(), lens.data_ptr(), 16384, None,
                                             roots2.data_ptr(), dn.data_ptr(), dno.data_ptr(),
                                             dm.data_ptr(), dt.data_ptr(), dto.data_ptr(),
                                             dbs.data_ptr(), tree_bs, out2.data_ptr(),
                                             t1.value - 1, None, ctypes.byref(r2),
                                             ctypes.byref(t2), None))


def test_post_tree_device_keyed_cid_and_ctext(gpu, O):
    """The one call with a keyed CID and both ctext outputs (the blobs' and
    the tree blob's) against the three calls with the same key, after a
    call that failed on a short line buffer (the next call starts clean):
    roots, lines, every ctext byte and the tree root."""
    import ctypes
    import random
    import torch
    from glfs_amd import _native as N
    n, tree_bs = 5000, 64 * 1024
    rng = random.Random(77)
    lens_h = [rng.choice([0, 1, 100, 4096, 9000, 16384]) for _ in range(n)]
    offs_h, o = [], 0
    for ln in lens_h:
        offs_h.append(o)
        o += (ln + 15) // 16 * 16
    data = torch.empty(o + 64, dtype=torch.uint8, device="cuda")
    N.check(N.lib.glfsx_fill_splitmix_device(data.data_ptr(), 0, o + 8 - o % 8, 3, None))
    names = [b"k%05d" % i for i in range(n)]
    types = [b"blob"] * n
    modes = [0o644] * n
    bss = [2 * MIB] * n
    offs = torch.tensor(offs_h, dtype=torch.int64, device="cuda")
    lens = torch.tensor(lens_h, dtype=torch.int64, device="cuda")
    dn, dno, dm, dt, dto, _, dbs = _tree_inputs(torch, names, types, modes, lens_h, bss)
    bsalt, tsalt = O.derive_key(bytes(32), b"blob"), O.derive_key(bytes(32), b"tree")
    key = bytes(range(40, 72))
    cap = 300 * n + 4096
    torch.cuda.synchronize()
    ct1 = torch.zeros(o + 64, dtype=torch.uint8, device="cuda")
    roots1 = torch.zeros(64 * n, dtype=torch.uint8, device="cuda")
    N.check(N.lib.glfsx_post_blobs_device(2 * MIB, bsalt, key, data.data_ptr(), offs.data_ptr(),
                                          lens.data_ptr(), n, 16384, ct1.data_ptr(),
                                          roots1.data_ptr(), None))
    out1 = torch.zeros(cap, dtype=torch.uint8, device="cuda")
    t1 = ctypes.c_uint64()
    N.check(N.lib.glfsx_tree_encode_device(n, dn.data_ptr(), dno.data_ptr(), dm.data_ptr(),
                                           dt.data_ptr(), dto.data_ptr(), roots1.data_ptr(),
                                           lens.data_ptr(), dbs.data_ptr(), out1.data_ptr(),
                                           cap, None, ctypes.byref(t1), None))
    tct1 = torch.zeros(t1.value + 64, dtype=torch.uint8, device="cuda")
    r1 = N.glfsx_root()
    N.check(N.lib.glfsx_create_device(tree_bs, tsalt, key, out1.data_ptr(), t1.value,
                                      tct1.data_ptr(), ctypes.byref(r1), None, None))
    torch.cuda.synchronize()
    ct2 = torch.zeros(o + 64, dtype=torch.uint8, device="cuda")
    roots2 = torch.zeros(64 * n, dtype=torch.uint8, device="cuda")
    out2 = torch.zeros(cap, dtype=torch.uint8, device="cuda")
    tct2 = torch.zeros(t1.value + 64, dtype=torch.uint8, device="cuda")
    r2, t2 = N.glfsx_root(), ctypes.c_uint64()

    def one_call(cap2):
        return N.lib.glfsx_post_tree_device(n, 2 * MIB, bsalt, tsalt, key, data.data_ptr(),
                                            offs.data_ptr(), lens.data_ptr(), 16384,
                                            ct2.data_ptr(), roots2.data_ptr(), dn.data_ptr(),
                                            dno.data_ptr(), dm.data_ptr(), dt.data_ptr(),
                                            dto.data_ptr(), dbs.data_ptr(), tree_bs,
                                            out2.data_ptr(), cap2, tct2.data_ptr(),
                                            ctypes.byref(r2), ctypes.byref(t2), None)
    with pytest.raises(N.GlfsxError):
        N.check(one_call(t1.value - 1))
    N.check(one_call(cap))
    torch.cuda.synchronize()
    assert t2.value == t1.value
    assert torch.equal(roots1, roots2)
    assert torch.equal(out1[:t1.value], out2[:t2.value])
    assert torch.equal(ct1[:o], ct2[:o])
    assert torch.equal(tct1[:t1.value], tct2[:t1.value])
    assert bytes(r2.ref) == bytes(r1.ref)
    i = 4321
    want_root, _, _, _ = O.create(bytes(data[offs_h[i]:offs_h[i] + lens_h[i]].cpu().numpy()
                                        .tobytes()), 2 * MIB, salt=bsalt, cid_key=key,
                                  closed_form=True)
    assert bytes(roots2[64 * i:64 * i + 64].cpu().numpy().tobytes()) == want_root

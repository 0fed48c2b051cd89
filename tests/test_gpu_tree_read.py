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

"""The reference's own Go tests for the write path and its neighbours,
restated against the GPU path (same inputs where the Go test's inputs are
reproducible, splitmix bytes where they come from math/rand -- Go's RNG
stream is not reproducible here).  Each test names the Go test it
mirrors; results are additionally checked against the oracle."""
import random

import pytest

pytestmark = pytest.mark.gpu

KIB, MIB = 1 << 10, 1 << 20


def test_ref_post_get(gpu, O):
    """bigblob/ref_test.go:13-25 TestRefPostGet: post "test data" with a zero
    salt into a 1 KiB store, getF gives it back."""
    from glfs_amd import bigblob
    m = bigblob.Machine()
    s = bigblob.MemStore(1 << 10)
    ref = m.post(s, bytes(32), b"test data")
    assert m.get_f(s, ref) == b"test data"
    want, ct = O.post(bytes(32), b"test data")
    assert ref.marshal_binary() == want and s.get(ref.cid) == ct


def test_ref_post_empty_and_keyed(gpu, O):
    """post of the empty message (blob.go:187-189 posts post(indexSalt, nil))
    and with a keyed store hash."""
    from glfs_amd import bigblob
    m = bigblob.Machine()
    s = bigblob.MemStore(1 << 10)
    salt = bytes(range(32))
    assert m.post(s, salt, b"").marshal_binary() == O.post(salt, b"")[0]
    key = bytes(range(64, 96))
    data = O.fill_splitmix(1000, 3)
    assert m.post(s, salt, data, cid_key=key).marshal_binary() == \
        O.post(salt, data, cid_key=key)[0]


def test_ref_marshal(gpu):
    """bigblob/ref_test.go:27-40 TestRefMarshal on a GPU-posted ref."""
    from glfs_amd import bigblob
    ref = bigblob.Machine().post(bigblob.MemStore(1 << 10), bytes(32), b"test data")
    data = ref.marshal_binary()
    assert len(data) == bigblob.REF_SIZE
    assert bigblob.Ref.from_bytes(data) == ref


def test_create_file(gpu, O):
    """bigblob/blob_test.go:47-65 TestCreateFile: 3 MiB at the store's 1 MiB
    max (NewMachine: block size 0 = MaxSize) -> Size 3 MiB, the root exists,
    exactly 4 blobs (3 data + 1 index)."""
    from glfs_amd import bigblob
    s = bigblob.MemStore(1 << 20)
    data = O.fill_splitmix(3 * MIB, 0)
    root = bigblob.Machine().create(s, None, data)
    assert root.size == 3 * MIB
    assert bigblob.exists_unit(s, root.ref.cid)
    assert len(s) == 4
    assert root.ref.marshal_binary() == O.create(data, MIB, salt=None)[0]


_BS = 1 << 10
_BF = _BS // 64
CREATE_READ_SIZES = [0, 1, 100, _BS // 2, _BS, _BS * 2, _BS * 2 - 1, _BS * 2 + 1,
                     _BS * _BF, _BS * _BF + 1, _BS * _BF - 1,
                     _BS * _BF * _BF, _BS * _BF * _BF + 1, _BS * _BF * _BF - 1]


@pytest.mark.parametrize("size", CREATE_READ_SIZES)
def test_create_read(gpu, O, size):
    """bigblob/blob_test.go:67-106 TestCreateRead, its 14 sizes.  As written,
    testCreateRead ignores blockSize (NewMachine(), 1 MiB store: every size is
    one block); both that and the intended 1 KiB block size (depth up to 3)
    are run: Create, read back through the Reader, root vs the oracle."""
    from glfs_amd import bigblob
    data = O.fill_splitmix(size, 0)
    for bs_opt, store_max in ((0, 1 << 20), (_BS, 1 << 20)):
        s = bigblob.MemStore(store_max)
        m = bigblob.Machine(bs_opt)
        root = m.create(s, None, data)
        bs = bs_opt or store_max
        assert (root.size, root.block_size) == (size, bs)
        assert m.new_reader(s, root).read() == data
        want, _, _, posts = O.create(data, bs, salt=None, store_max=store_max)
        assert root.ref.marshal_binary() == want
        assert len(s.log) == len(posts)


def test_glfs_sync(gpu):
    """glfs_test.go:16-42 TestSync: an empty blob and a tree of three blobs
    (two with content, one empty) sync into an empty store; everything the
    tree references arrives; a second Sync posts nothing."""
    from glfs_amd import bigblob, glfs
    src = bigblob.MemStore(glfs.DEFAULT_BLOCK_SIZE)
    empty = glfs.post_blob(src, b"")
    tree = glfs.post_tree_map(src, {"a": glfs.post_blob(src, b"hello"),
                                    "b": glfs.post_blob(src, b"world"),
                                    "c": glfs.post_blob(src, b"")})
    for ref in (empty, tree):
        dst = bigblob.MemStore(glfs.DEFAULT_BLOCK_SIZE)
        glfs.sync(dst, src, ref)
        assert bigblob.exists_unit(dst, ref.root.ref.cid)
        n = len(dst.log)
        glfs.sync(dst, src, ref)
        assert len(dst.log) == n
    assert set(dst.blobs) == set(src.blobs)   # the tree reaches every blob
    got = glfs.Machine().get_tree_slice(dst, tree)
    assert [e.name for e in got] == ["a", "b", "c"]
    assert glfs.Machine().get_blob_bytes(dst, got[1].ref, 100) == b"world"
    with pytest.raises(ValueError):
        glfs.sync(dst, src, glfs.Ref("nope", empty.root))


def _tree_with_dirs():
    from glfs_amd import bigblob, glfs
    s = bigblob.MemStore(glfs.DEFAULT_BLOCK_SIZE)
    blob = glfs.post_blob(s, b"")       # tree_test.go:143-147 blobRef
    m1 = {"dir1/file1.1": blob, "dir1/file1.2": blob, "dir2/file2.1": blob}
    return s, m1, glfs.post_tree_map(s, m1)


def test_post_tree_from_entries(gpu):
    """tree_test.go:15-29 TestPostTreeFromEntries: every path resolves to a
    blob through GetAtPath."""
    from glfs_amd import glfs
    s, m1, ref = _tree_with_dirs()
    for k in m1:
        got = glfs.get_at_path(s, ref, k)
        assert got.type == glfs.TYPE_BLOB and got == m1[k]
    assert glfs.get_at_path(s, ref, "/dir1/").type == glfs.TYPE_TREE
    assert glfs.get_at_path(s, ref, "") == ref


def test_tree_no_ent(gpu):
    """tree_test.go:31-44 TestTreeNoEnt and errors_test TestIsErrNoEnt."""
    from glfs_amd import glfs, tree as T
    s, _, ref = _tree_with_dirs()
    with pytest.raises(T.ErrNoEnt) as ei:
        glfs.get_at_path(s, ref, "should-not-exist")
    assert T.is_err_no_ent(ei.value) and ei.value.name == "should-not-exist"
    with pytest.raises(T.ErrNoEnt):
        glfs.get_at_path(s, ref, "dir1/file1.9")
    with pytest.raises(T.TreeError, match="subpath of type tree"):
        glfs.get_at_path(s, ref, "dir1/file1.1/x")
    assert T.is_err_no_ent(T.ErrNoEnt("x")) and not T.is_err_no_ent(ValueError())


def test_data_not_found(gpu):
    """tree_test.go:84-97 TestDataNotFound: with the tree blob deleted,
    GetAtPath fails with the store's not-found error for that CID."""
    from glfs_amd import bigblob, glfs
    s = bigblob.MemStore(glfs.DEFAULT_BLOCK_SIZE)
    ref = glfs.post_tree_map(s, {k: glfs.post_blob(s, b"hello " + k.encode())
                                 for k in "abc"})
    s.delete([ref.root.ref.cid])
    with pytest.raises(bigblob.ErrNotFound) as ei:
        glfs.get_at_path(s, ref, "a")
    assert ei.value.cid == ref.root.ref.cid


def test_post_many_random(gpu, O):
    """post() over random sizes and salts (ref.go:98-111) vs the oracle."""
    from glfs_amd import bigblob
    m = bigblob.Machine()
    s = bigblob.MemStore(4 * MIB)
    rng = random.Random(8)
    for _ in range(25):
        n = rng.choice([0, 1, 63, 64, 65, 1023, 1024, 1025, rng.randrange(1, 3 * MIB)])
        salt = rng.randbytes(32)
        data = O.fill_splitmix(n, n ^ 77)
        ref = m.post(s, salt, data)
        want, ct = O.post(salt, data)
        assert ref.marshal_binary() == want and s.get(ref.cid) == ct, n

"""The store boundary (ref.go:103 s.Post; blobcache MemStore [ext]): the
native store of the C-ABI with a pre-hashed Post (trust the GPU CID, verify
a sample in parity mode) and a re-hashing Post (today's MemStore behaviour).
Host-only parts run without a GPU; the Writer into the store is -m gpu."""
import pytest

from glfs_amd import bigblob

MIB = 1 << 20


def _refs(O, n, seed=1):
    out = []
    for i in range(n):
        data = O.fill_splitmix(1000 + 37 * i, seed + i)
        ref, ct = O.post(bytes(32), data)
        out.append((ref, ct))
    return out


def test_trusting_post_get_exists(O):
    s = bigblob.NativeStore(MIB, "trust")
    posts = _refs(O, 20)
    for ref, ct in posts:
        s.post(ct, ref)
    s.post(posts[0][1], posts[0][0])                   # re-post: idempotent
    assert len(s) == 20
    st = s.stats()
    assert st["posts"] == 21 and st["rehashed"] == 0
    for ref, ct in posts:
        assert s.exists(ref[:32]) and s.get(ref[:32]) == ct
    assert not s.exists(bytes(32))
    with pytest.raises(bigblob.ErrNotFound):
        s.get(bytes(32))
    # a trusting store takes whatever CID it is given (that is the point)
    s.post(b"xyz", bytes(range(64)))
    assert s.get(bytes(range(32))) == b"xyz"


def test_hashing_and_verifying_posts(O):
    posts = _refs(O, 10, seed=7)
    h = bigblob.NativeStore(MIB, "hash")
    for ref, ct in posts:
        h.post(ct, ref)
    assert h.stats()["rehashed"] == 10
    bad = bytearray(posts[3][0])
    bad[5] ^= 1
    with pytest.raises(bigblob.StoreError):
        h.post(posts[3][1], bytes(bad))
    v = bigblob.NativeStore(MIB, "trust", verify_every=2)
    with pytest.raises(bigblob.StoreError):            # post 0 is verified
        v.post(posts[3][1], bytes(bad))
    v.post(posts[4][1], bytes(bad))                    # post 1 is not
    # keyed store CIDs
    key = bytes(range(5, 37))
    k = bigblob.NativeStore(MIB, "hash", cid_key=key)
    data = O.fill_splitmix(3000, 3)
    ref, ct = O.post(bytes(32), data, cid_key=key)
    k.post(ct, ref)
    assert k.exists(ref[:32])


def test_max_size_and_keep_data(O):
    s = bigblob.NativeStore(1024, "trust", keep_data=False)
    ref, ct = O.post(bytes(32), O.fill_splitmix(1000, 1))
    s.post(ct, ref)
    assert s.exists(ref[:32]) and s.get(ref[:32]) == b""
    with pytest.raises(bigblob.StoreError):
        s.post(bytes(1025), bytes(64))


@pytest.mark.gpu
@pytest.mark.parametrize("mode,verify", [("trust", 0), ("trust", 3), ("hash", 0)])
def test_writer_into_native_store(gpu, O, mode, verify):
    """The Writer delivers every Post to the native store as a C call; the
    root and every stored ctext equal the oracle's, and the blob reads back
    through the GPU decrypt."""
    bs = 64 << 10
    data = O.fill_splitmix(200 * bs + 5, 12)
    want_root, _, _, want_posts = O.create(data, bs)
    s = bigblob.NativeStore(bs, mode, verify_every=verify)
    root = bigblob.Machine(bs).create(s, None, data)
    assert root.ref.marshal_binary() == want_root
    assert len(s) == len(want_posts)
    for _, ref, _, ct in want_posts:
        assert s.get(ref[:32]) == ct
    st = s.stats()
    assert st["rehashed"] == (len(want_posts) if mode == "hash" else
                              (-(-len(want_posts) // verify) if verify else 0))
    assert bigblob.read_all(s, root) == data

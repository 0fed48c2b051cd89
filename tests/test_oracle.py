"""Pin the CPU oracle (oracle/) before trusting it (CPU-only).

  * BLAKE3 (lukechampine.com/blake3 v1.2.1 [ext]) against upstream C BLAKE3
    1.8.2 in libclang-cpp.so and published vectors;
  * ChaCha20 (golang.org/x/crypto chacha20 [ext]) against OpenSSL, libsodium
    and RFC 8439 A.1;
  * the bigblob layer against the reference's own structural tests
    (bigblob/blob_test.go TestDepth / TestCreateFile) and SURVEY.md's anchors
    (an independent restatement of blob.go/ref.go).
"""
import random

import pytest

import refimpl as R

B3_EMPTY = "af1349b9f5f9a1a6a0404dea36dcc9499bcb25c9adc112b7cc9a93cae41f3262"
B3_ABC = "6437b3ac38465133ffb63b75273a8db548c558465d79db03fd359c6cd5bd9d85"
# RFC 8439 A.1 test vector #1: key 0, nonce 0, counter 0 keystream
RFC8439_A1_1 = ("76b8e0ada0f13d90405d6ae55386bd28bdd219b8a08ded1aa836efcc8b770dc7"
                "da41597c5157488d7724e03fb8d84a376a43b8f41518a11cc387b669b2ee6586")


def test_blake3_published(O):
    assert O.blake3(b"").hex() == B3_EMPTY
    assert O.blake3(b"abc").hex() == B3_ABC


@pytest.mark.skipif(R.blake3_lib() is None, reason="libclang-cpp BLAKE3 absent")
def test_blake3_vs_upstream_c(O):
    rng = random.Random(5)
    key = bytes(rng.randrange(256) for _ in range(32))
    sizes = [0, 1, 63, 64, 65, 1023, 1024, 1025, 2047, 2048, 2049, 3 * 1024 + 7,
             4096, 8191, 8192, 8193, 16 * 1024 + 1, 31 * 1024, 65536, 100_003]
    for n in sizes:
        data = bytes(rng.randrange(256) for _ in range(n))
        assert O.blake3(data) == R.blake3(data), n
        assert O.blake3(data, key) == R.blake3(data, key), n
        # XOF beyond one output block
        assert O.blake3(data, key, 131) == R.blake3(data, key, 131), n


def test_chacha20_rfc8439(O):
    assert O.chacha20_xor(bytes(64), bytes(32)).hex() == RFC8439_A1_1


@pytest.mark.skipif(R.openssl_lib() is None, reason="libcrypto absent")
def test_chacha20_vs_openssl_and_sodium(O):
    rng = random.Random(6)
    for n in [0, 1, 63, 64, 65, 127, 128, 129, 1000, 4096, 70_001]:
        key = bytes(rng.randrange(256) for _ in range(32))
        data = bytes(rng.randrange(256) for _ in range(n))
        for ctr in (0, 1, 1000):
            ours = O.chacha20_xor(data, key, bytes(12), ctr)
            assert ours == R.chacha20_xor(data, key, bytes(12), ctr)
            if R.sodium_lib() is not None:
                assert ours == R.sodium_chacha20_xor(data, key, bytes(12), ctr)


def test_survey_anchors(O):
    """SURVEY.md 8c anchors (an independent restatement of the Go path)."""
    z = bytes(32)
    assert O.derive_key(z, b"raw").hex() == \
        "64d0a4731fc12b70a7a6256a4f8cb0c3f3995ec9c119fe15671e2d6429e14f05"
    assert O.derive_key(z, b"index").hex() == \
        "3cf865a69db774075f598e07277b30fb5094841c032d0085861a72737aeb84c9"
    blob = O.derive_key(z, b"blob")
    assert blob.hex() == "0a08c904a5c09e4147a540cdd557af8718830d2dfc1d9e16880602801f910afa"
    tree = O.derive_key(z, b"tree")
    assert tree.hex() == "b8d78833bea07389354d1fde49eba54246b6366e07044bff7f5819074a8b743c"
    root, size, bs, posts = O.create(b"test data", 2 << 20, salt=blob)
    assert root[:32].hex() == "c46ac4e44a328b9c07cba45eddb89b635fa44746823f4f5d3f01e39f52a6c851"
    assert root[32:].hex() == "d0d02185d4646a367978c907c9b04fd4b7c536467d9c1882a67b2079b8c9841d"
    assert (size, bs, len(posts)) == (9, 2 << 20, 1)
    root, *_ = O.create(b"", 2 << 20, salt=blob)
    assert root[:32].hex() == B3_EMPTY
    assert root[32:].hex() == "a00277bdf712846b278e91f8493738de216c18b1f2c1a58b0d52562aa40eb589"
    root, *_ = O.create(O.mod251(4096), 2 << 20, salt=blob)
    assert root[:32].hex() == "eab5d7f27316ee27cbf25fc59dc179a7cdc73fde2d904119ba4431c5d97cb29d"
    root, _, _, posts = O.create(O.mod251((2 << 20) + 1), 2 << 20, salt=blob)
    assert root[:32].hex() == "93999f19c8a9b2ef781bf039d394c4aa7561f7190e42f1bb375fffb7e65b9da1"
    assert len(posts) == 3
    root, _, _, posts = O.create(O.mod251(3 << 20), 1 << 20, salt=None)
    assert root[:32].hex() == "ee2fb783ba792823e9f1404f75e3aed9eaaaa8871b592cccd5073aff27ab313a"
    root, *_ = O.create(O.mod251(1024 * 16 * 16 + 1), 1024, salt=None)
    assert root[:32].hex() == "175173c395b557e1e59521652ffef0fd878f5dbc0c9c43c59aafbaf9b1e589eb"


def test_depth_table(O):
    """bigblob/blob_test.go:16-45 TestDepth."""
    bs = 1 << 10
    bf = bs // 64
    table = [(1 << 10, 0, 0), (1 << 10, 1 << 10, 0), (1 << 10, (1 << 10) + 1, 1),
             (1 << 10, 1 << 12, 1), (1 << 10, 8192, 1),
             (bs, bs * bf - 1, 1), (bs, bs * bf, 1), (bs, bs * bf + 1, 2),
             (bs, bs * bf * bf - 1, 2), (bs, bs * bf * bf, 2), (bs, bs * bf * bf + 1, 3),
             (bs, bs * bf ** 3 - 1, 3), (bs, bs * bf ** 3, 3), (bs, bs * bf ** 3 + 1, 4)]
    for b, size, want in table:
        assert O.depth(size, b) == want, (b, size)


def test_create_file_four_blobs(O):
    """bigblob/blob_test.go:47-65: 3 MiB at 1 MiB blocks -> 3 data + 1 index."""
    root, size, bs, posts = O.create(O.fill_splitmix(3 << 20, 0), 1 << 20, salt=None,
                                     store_max=1 << 20)
    assert size == 3 << 20
    assert len({p[1][:32] for p in posts}) == 4
    assert [p[0] for p in posts] == [0, 0, 0, 1]
    assert posts[-1][1] == root


def test_writer_panics(O):
    """blob.go:90-95; examples/write-read-blob posts into a 1 MiB store with the
    2 MiB glfs default and panics at reference HEAD (SURVEY checklist)."""
    with pytest.raises(O.WriterPanic, match="2097152 > maxSize 1048576"):
        O.create(b"test data", 2 << 20, store_max=1 << 20)
    with pytest.raises(O.WriterPanic, match="< 128"):
        O.create(b"x", 127, store_max=1 << 20)


@pytest.mark.parametrize("bs", [128, 1000, 1024])
def test_streaming_equals_closed_form(O, bs):
    bf = bs // 64
    rng = random.Random(bs)
    sizes = {0, 1, bs - 1, bs, bs + 1, bf * bs - 1, bf * bs, bf * bs + 1,
             bf * bf * bs + bs + 3, rng.randrange(1, 40 * bs)}
    for n in sorted(sizes):
        data = O.fill_splitmix(n, n)
        a = O.create(data, bs, salt=None)
        b = O.create(data, bs, salt=None, closed_form=True)
        assert a[0] == b[0], n
        assert len(a[3]) == len(b[3]), n
        assert sorted(p[1] for p in a[3]) == sorted(p[1] for p in b[3]), n


def test_write_granularity_invariance(O):
    """io.Copy piece sizes (blob.go:120-133 recursion) do not change refs."""
    data = O.fill_splitmix(5000, 3)
    want = O.create(data, 1024, salt=None)
    rng = random.Random(7)
    for _ in range(5):
        pieces = []
        left = len(data)
        while left:
            k = min(left, rng.choice([1, 7, 100, 1023, 1024, 1025, 3000]))
            pieces.append(k)
            left -= k
        got = O.create(data, 1024, salt=None, chunks=pieces)
        assert got[0] == want[0]
        assert [(p[0], p[1]) for p in got[3]] == [(p[0], p[1]) for p in want[3]]


def test_simd_cpu_baseline_same_refs(O):
    """bench's second CPU baseline (upstream BLAKE3 C + OpenSSL ChaCha20,
    oracle/cpu_simd.c) computes the same refs and ctext as the scalar port."""
    import ctypes
    L = O.lib()
    n, bs = 5 * 1024 * 1024 + 777, 1 << 20
    data = O.fill_splitmix(n, 4)
    salt = O.derive_key(bytes(32), b"raw")
    nb = -(-n // bs)
    a, b = ctypes.create_string_buffer(64 * nb), ctypes.create_string_buffer(64 * nb)
    ca, cb = ctypes.create_string_buffer(n), ctypes.create_string_buffer(n)
    L.oracle_post_batch(a, ca, salt, data, n, bs, None, 2)
    rc = L.oracle_post_batch_simd(b, cb, salt, data, n, bs, None, 3)
    if rc == -1:
        pytest.skip("libclang-cpp BLAKE3 or libcrypto absent")
    assert a.raw == b.raw and ca.raw == cb.raw
    # the Go path's mix (SIMD BLAKE3 + scalar ChaCha20): bench's cpu_baseline.value
    g, cg = ctypes.create_string_buffer(64 * nb), ctypes.create_string_buffer(n)
    assert L.oracle_post_batch_gomix(g, cg, salt, data, n, bs, None, 2) == 0
    assert a.raw == g.raw and ca.raw == cg.raw

"""Host logic of the tree path (tree.go), no GPU: Go json.Encoder line bytes,
CleanPath, ordering, lookup, and decoding.  The expected strings are written
out by hand from Go's encoding rules (encoding/json, go 1.25)."""
import pytest

from glfs_amd import bigblob, glfs, tree as T


def _ref(ty="blob", size=9, bs=2 << 20, c=0x11, d=0x22):
    return glfs.Ref(ty, bigblob.Root(bigblob.Ref(bytes([c]) * 32, bytes([d]) * 32), size, bs))


@pytest.mark.parametrize("s,want", [
    ("plain", '"plain"'),
    ('q"b\\s', '"q\\"b\\\\s"'),
    ("<a&b>", '"\\u003ca\\u0026b\\u003e"'),
    ("\n\r\t\b\f", '"\\n\\r\\t\\b\\f"'),
    ("\x00\x01\x1f", '"\\u0000\\u0001\\u001f"'),
    ("\u2028\u2029", '"\\u2028\\u2029"'),
    ("é日本\U0001F600", '"é日本\U0001F600"'),
    ("bad\udc80", '"bad\\ufffd"'),
    ("a\udcff\udc80b", '"a\\ufffd\\ufffdb"'),
    ("\x7f", '"\x7f"'),
])
def test_go_json_string(s, want):
    assert T.go_json_string(s) == want


def test_entry_line_bytes():
    te = T.TreeEntry("a<b>.txt", 0o644, _ref())
    want = ('{"name":"a\\u003cb\\u003e.txt","mode":420,"ref":{"type":"blob","cid":"'
            + "11" * 32 + '","dek":"' + "22" * 32 + '","size":9,"blockSize":2097152}}\n')
    assert T.entry_json_line(te) == want.encode()
    td = T.TreeEntry("dir", T.get_file_mode(_ref("tree")), _ref("tree", 100, 2 << 20))
    assert b'"mode":2147484141,' in T.entry_json_line(td)  # 0755 | os.ModeDir


def test_cid_json_pluggable():
    import base64
    enc = lambda c: '"' + base64.urlsafe_b64encode(c).decode().rstrip("=") + '"'
    dec = lambda v: base64.urlsafe_b64decode(v + "=" * (-len(v) % 4))
    te = T.TreeEntry("x", 0o644, _ref(c=0xAB))
    line = T.entry_json_line(te, enc)
    assert T.read_tree_bytes(line, dec) == [te]


@pytest.mark.parametrize("x,want", [
    ("", ""), (".", ""), ("/", ""), ("a", "a"), ("a/", "a"), ("/a/b/", "a/b"),
    ("a//b", "a/b"), ("a/./b", "a/b"), ("a/../b", "b"), ("a/..", ""),
    ("../a", "../a"), ("/../a", "a"), ("a/b/../../..", ".."), ("./a/./", "a"),
])
def test_clean_path(x, want):
    assert T.clean_path(x) == want


def test_validate_and_names():
    assert T.is_valid_name("a") and not T.is_valid_name("") and not T.is_valid_name("a/b")
    with pytest.raises(T.TreeError, match="not properly cleaned"):
        T.TreeEntry("a/", 0o644, _ref()).validate()
    with pytest.raises(T.TreeError, match="cannot be empty"):
        T.TreeEntry("", 0o644, _ref()).validate()
    ents = [T.TreeEntry(n, 0o644, _ref()) for n in ["b", "a", "B", "é", "a0"]]
    T.sort_tree_entries(ents)
    assert [e.name for e in ents] == ["B", "a", "a0", "b", "é"]  # byte order
    T.validate_tree_entries(ents)
    assert T.lookup(ents, "a0").name == "a0" and T.lookup(ents, "zz") is None
    with pytest.raises(T.TreeError, match="not sorted"):
        T.validate_tree_entries(ents[::-1])
    with pytest.raises(T.TreeError, match="duplicate"):
        T.validate_tree_entries([ents[0], ents[0]])


def test_read_tree_bytes_roundtrip_and_order():
    ents = [T.TreeEntry("%07d" % i, 0o644, _ref(size=i, c=i)) for i in range(50)]
    data = b"".join(T.entry_json_line(e) for e in ents)
    assert T.read_tree_bytes(data) == ents
    bad = T.entry_json_line(ents[1]) + T.entry_json_line(ents[0])
    with pytest.raises(T.TreeError, match="out of order"):
        T.read_tree_bytes(bad)
    assert T.read_tree_bytes(b"") == []


def test_native_encoder_matches_python():
    """glfsx_tree_encode (host C++, multi-threaded; no GPU) writes the same
    bytes as entry_json_line for every escaping class, line by line."""
    import random
    rng = random.Random(7)
    pool = ["plain", "<a&b>", "\n\r\t\b\f\x00\x1f\x7f", " x ", "é日本\U0001F600",
            "bad\udc80\udcff", "q\"b\\s", "", "%07d" % 5, "\udced\udca0\udc80"]
    ents = []
    for i in range(20000):
        name = rng.choice(pool) + str(i) + rng.choice(pool)
        ty = rng.choice(["blob", "tree", "t<&>", " "])
        r = glfs.Ref(ty, bigblob.Root(bigblob.Ref(rng.randbytes(32), rng.randbytes(32)),
                                      rng.randrange(1 << 62), rng.choice([128, 2 << 20])))
        ents.append(T.TreeEntry(name, rng.choice([0o644, T.MODE_TREE, 0]), r))
    data, ends = T.encode_lines(ents)
    want = [T.entry_json_line(e) for e in ents]
    assert data == b"".join(want)
    acc = 0
    for ln, e in zip(want, ends):
        acc += len(ln)
        assert e == acc
    assert T.encode_lines([]) == (b"", [])

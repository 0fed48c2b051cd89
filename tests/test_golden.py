"""The oracle reproduces the committed fixtures (tests/golden/, CPU-only)."""
import json
import os

import pytest

import refimpl as R

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name):
    with open(os.path.join(HERE, name)) as f:
        return json.load(f)


def data_for(O, gen, n):
    if gen == "mod251":
        return O.mod251(n)
    if gen.startswith("splitmix:"):
        return O.fill_splitmix(n, int(gen.split(":")[1]))
    if gen.startswith("literal:"):
        return gen.split(":", 1)[1].encode()
    raise ValueError(gen)


def test_primitive_vectors(O):
    p = load("primitives.json")
    key = bytes.fromhex(p["blake3_key"])
    for v in p["blake3"]:
        d = data_for(O, v["gen"], v["len"])
        assert O.blake3(d).hex() == v["hash"]
        assert O.blake3(d, key).hex() == v["keyed_hash"]
        if R.blake3_lib() is not None:
            assert R.blake3(d).hex() == v["hash"]
    for v in p["chacha20"]:
        d = data_for(O, v["gen"], v["len"])
        ct = O.chacha20_xor(d, bytes.fromhex(v["key"]), bytes.fromhex(v["nonce"]),
                            v["counter"])
        assert ct.hex() == v["ctext"]


CASES = load("bigblob.json")["cases"]


@pytest.mark.parametrize("c", [c for c in CASES if c["size"] <= (4 << 20) + 1],
                         ids=lambda c: c["name"])
def test_bigblob_vectors(O, c):
    data = data_for(O, c["gen"], c["size"])
    salt = bytes.fromhex(c["salt"]) if c["salt"] else None
    root, size, bs, posts = O.create(data, c["block_size"], salt=salt)
    assert root[:32].hex() == c["root"]["cid"]
    assert root[32:].hex() == c["root"]["dek"]
    assert (size, bs) == (c["root"]["size"], c["root"]["blockSize"])
    assert len(posts) == c["n_posts"]
    assert O.depth(c["size"], c["block_size"]) == c["depth"]
    if "posts" in c:
        assert [[k, n, r[:32].hex(), r[32:].hex()] for k, r, n, _ in posts] == c["posts"]


def test_salts(O):
    s = load("bigblob.json")["salts"]
    z = bytes(32)
    for ty in ("blob", "tree"):
        ts = O.derive_key(z, ty.encode())
        assert ts.hex() == s[ty]["type_salt"]
        assert O.derive_key(ts, b"raw").hex() == s[ty]["raw_salt"]
        assert O.derive_key(ts, b"index").hex() == s[ty]["index_salt"]
    assert O.derive_key(z, b"raw").hex() == s["nil"]["raw_salt"]

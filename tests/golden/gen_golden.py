"""Generate tests/golden/*.json (committed fixtures).

Inputs are synthetic (the reference's own tests use Go's math/rand stream,
which cannot be reproduced without Go, and hold no golden CIDs/DEKs -- SURVEY
4/8c).  Expected outputs come from the CPU oracle (oracle/), and every
primitive value is cross-checked here against independent libraries in the
image (upstream C BLAKE3 1.8.2 in libclang-cpp.so, OpenSSL EVP_chacha20)
before being written.  Bigblob-level vectors follow bigblob/blob.go:85-206
(streaming writer) and are cross-checked against the closed-form builder.

Run:  python tests/golden/gen_golden.py
"""
from __future__ import annotations

import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(HERE))

from oracle import oracle as O  # noqa: E402
import refimpl as R  # noqa: E402

KIB, MIB = 1 << 10, 1 << 20


def gen_data(gen: str, n: int) -> bytes:
    if gen == "mod251":
        return O.mod251(n)
    if gen.startswith("splitmix:"):
        return O.fill_splitmix(n, int(gen.split(":")[1]))
    if gen.startswith("literal:"):
        return gen.split(":", 1)[1].encode()
    raise ValueError(gen)


def primitives() -> dict:
    out = {"blake3": [], "chacha20": []}
    key = bytes(range(32))
    for n in [0, 1, 63, 64, 65, 1023, 1024, 1025, 2048, 2049, 3072, 3073, 4096,
              4097, 5120, 5121, 6144, 6145, 7168, 7169, 8192, 8193, 16384, 31744,
              102400]:
        data = O.mod251(n)
        plain = O.blake3(data)
        keyed = O.blake3(data, key)
        assert plain == R.blake3(data), n
        assert keyed == R.blake3(data, key), n
        out["blake3"].append({"gen": "mod251", "len": n, "hash": plain.hex(),
                              "keyed_hash": keyed.hex()})
    for n, ctr in [(0, 0), (1, 0), (63, 0), (64, 0), (65, 0), (1000, 0), (64, 1),
                   (129, 7)]:
        data = O.mod251(n)
        ct = O.chacha20_xor(data, key, bytes(12), ctr)
        assert ct == R.chacha20_xor(data, key, bytes(12), ctr), n
        out["chacha20"].append({"gen": "mod251", "len": n, "key": key.hex(),
                                "nonce": bytes(12).hex(), "counter": ctr,
                                "ctext": ct.hex()})
    out["blake3_key"] = key.hex()
    return out


def case(name: str, gen: str, size: int, bs: int, salt: bytes | None,
         store_max: int | None = None, keep_posts: bool = True) -> dict:
    data = gen_data(gen, size)
    root, sz, rbs, posts = O.create(data, bs, salt=salt, store_max=store_max)
    croot, _, _, cposts = O.create(data, bs, salt=salt, closed_form=True)
    assert croot == root and len(cposts) == len(posts), name
    # verify every posted CID independently: CID = BLAKE3-256(ctext)
    for kind, ref, n, ct in posts:
        assert R.blake3(ct) == ref[:32]
    d = {"name": name, "gen": gen, "size": size, "block_size": bs,
         "salt": salt.hex() if salt is not None else None,
         "root": {"cid": root[:32].hex(), "dek": root[32:].hex(), "size": sz,
                  "blockSize": rbs},
         "n_posts": len(posts), "depth": O.depth(size, bs)}
    if keep_posts:
        d["posts"] = [[k, n, r[:32].hex(), r[32:].hex()] for k, r, n, _ in posts]
    return d


def bigblob_cases() -> list:
    zero = bytes(32)
    blob_salt = O.derive_key(zero, b"blob")
    tree_salt = O.derive_key(zero, b"tree")
    cases = []
    # glfs.PostBlob (typeSalt(blob), bs = DefaultBlockSize 2 MiB; glfs.go:12)
    G = 2 * MIB
    cases.append(case("glfs_config1_test_data", "literal:test data", 9, G, blob_salt))
    for n in [0, 1, 63, 64, 65, 1023, 1024, 1025, 4096]:
        cases.append(case(f"glfs_blob_mod251_{n}", "mod251", n, G, blob_salt))
    for n in [G - 1, G, G + 1]:
        cases.append(case(f"glfs_blob_mod251_{n}", "mod251", n, G, blob_salt))
    cases.append(case("glfs_tree_salt_4096", "mod251", 4096, G, tree_salt))
    # bigblob.Create with nil salt (blob.go:96-98), bs 1 MiB (blob_test.go:47-65)
    M = MIB
    cases.append(case("bigblob_3MiB_1MiB", "mod251", 3 * M, M, None))
    cases.append(case("bigblob_splitmix1_3MiB_1MiB", "splitmix:1", 3 * M + 12345, M, None))
    for n in [M - 1, M, M + 1]:
        cases.append(case(f"bigblob_mod251_{n}_1MiB", "mod251", n, M, None))
    # depth 1..4 at bs = 1 KiB, bf = 16 (blob_test.go:16-45 shapes)
    K = KIB
    for n in [0, 1, 100, 512, K, 2 * K - 1, 2 * K, 2 * K + 1, 16 * K - 1, 16 * K,
              16 * K + 1, 256 * K - 1, 256 * K, 256 * K + 1]:
        cases.append(case(f"bigblob_1KiB_mod251_{n}", "mod251", n, K, None,
                          keep_posts=n <= 16 * K + 1))
    cases.append(case("bigblob_1KiB_mod251_depth4", "mod251", 4096 * K + 1, K, None,
                      keep_posts=False))
    # odd block sizes (not a multiple of 64 / 1024)
    cases.append(case("bigblob_bs1000_splitmix7", "splitmix:7", 50_000, 1000, None))
    cases.append(case("bigblob_bs130_splitmix8", "splitmix:8", 3000, 130, None))
    cases.append(case("bigblob_bs4096_salted", "splitmix:9", 300_000, 4096,
                      bytes(range(32))))
    return cases


def main() -> None:
    prim = primitives()
    with open(os.path.join(HERE, "primitives.json"), "w") as f:
        json.dump(prim, f, indent=1)
    zero = bytes(32)
    salts = {}
    for ty in ["blob", "tree"]:
        ts = O.derive_key(zero, ty.encode())
        salts[ty] = {"type_salt": ts.hex(),
                     "raw_salt": O.derive_key(ts, b"raw").hex(),
                     "index_salt": O.derive_key(ts, b"index").hex()}
    salts["nil"] = {"raw_salt": O.derive_key(zero, b"raw").hex(),
                    "index_salt": O.derive_key(zero, b"index").hex()}
    cases = bigblob_cases()
    with open(os.path.join(HERE, "bigblob.json"), "w") as f:
        json.dump({"salts": salts, "cases": cases}, f, indent=1)
    print(f"wrote {len(cases)} bigblob cases")


if __name__ == "__main__":
    main()

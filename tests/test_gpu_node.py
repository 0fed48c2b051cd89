"""Latency-form posts at the 64 KiB span boundaries: index nodes
(ref.go:98-161 over index.go:33-38's zero-padded node), one-block Creates
and small batches of <= 4 MiB messages, which take the DEK pass (k_quad,
64 KiB per workgroup), the keystream and the CID pass.  Every ref and ctext
byte against the oracle at 1 / 2 / 64 spans, ragged and 1-byte last spans,
single- and multi-span messages in one launch, up to 256 workgroups and one
past, keyed CIDs, repeated launches, and index levels.  (Round 4 also tried
these posts as ONE launch whose span workgroups wait for the message's DEK
inside it, k_node: parity green on these cases but no faster -- DESIGN.md
section 4 -- so it was not kept.)
"""
import random

import pytest

from test_gpu_parity import _create_device, _post_batch_host, _torch, dev_bytes

pytestmark = pytest.mark.gpu

MIB = 1 << 20


@pytest.mark.parametrize("bs,total", [
    (4 * MIB, 4 * MIB),                 # one message, 64 spans
    (4 * MIB, 16 * MIB),                # 4 x 64 spans = 256 workgroups (the limit)
    (4 * MIB, 16 * MIB + 1),            # 5 messages: past the limit (other forms)
    (2 * MIB, 16 * MIB - 5),            # 8 x 32 spans, ragged last span
    (1_000_000, 4_000_123),             # spans not dividing the block, 5 messages
    (100_000, 100_001),                 # a 2-span message and a 1-byte one together
    (65536, 65536 * 7 + 1),             # single-span messages only
    (65537, 3 * 65537),                 # 2 spans each, the second of 1 byte
    (3 * MIB + 64, 3 * MIB + 64),       # a 64-byte last span
    (128, 1),
])
def test_node_post_vs_oracle(gpu, O, bs, total):
    rng = random.Random(bs * 31 + total)
    salt = bytes(rng.randrange(256) for _ in range(32))
    data = O.fill_splitmix(total, total + 17)
    n = (total + bs - 1) // bs
    want = [O.post(salt, data[j * bs:(j + 1) * bs]) for j in range(n)]
    for rep in range(2):   # a second launch on the same stream: a new epoch
        refs, ct = _post_batch_host(salt, data, bs)
        for j, (r, c) in enumerate(want):
            assert refs[64 * j:64 * j + 64] == r, (rep, j)
            assert ct[j * bs:j * bs + len(c)] == c, (rep, j)
    ck = bytes(range(7, 39))
    refs, _ = _post_batch_host(salt, data, bs, cid_key=ck)
    for j in sorted({0, n - 1}):
        assert refs[64 * j:64 * j + 64] == O.post(salt, data[j * bs:(j + 1) * bs],
                                                  cid_key=ck)[0], j


@pytest.mark.parametrize("bs,size", [(4096, 4096 * 64 * 5 + 3),   # 2 index levels
                                     (2 * MIB, 2 * MIB),           # one block: its ref
                                     (2 * MIB, 9 * MIB + 7),       # 5 blocks + the node
                                     (65536, 65536 * 1500 + 9)])   # 2 nodes, then the root
def test_node_create_device_vs_oracle(gpu, O, bs, size):
    torch = _torch()
    t = dev_bytes(torch, size, seed=size)
    root, posts = _create_device(torch, bs, t, size)
    want, _, _, want_posts = O.create(O.fill_splitmix(size, size), bs, salt=None,
                                      closed_form=True)
    assert root == want and posts == len(want_posts)

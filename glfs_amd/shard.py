"""Multi-GPU sharding of one bigblob write.

Each rank owns a contiguous range of data blocks that starts on a multiple
of bf = block_size/64, so the level-1 index nodes over its range are entirely
its own (bigblob/index.go:33-38, blob.go:165-182).  A rank posts its blocks
and its level-1 nodes on its GPU (glfsx_shard_device); the only exchange is
a gather of the level-1 refs (64 B per bf blocks: 256 B for a 64 GiB shard at
1 MiB blocks) after which one rank builds levels >= 2 and the root
(glfsx_root_from_level1).  No collective touches the data path.
"""
from __future__ import annotations

import ctypes
from typing import List, Tuple


def plan(size: int, block_size: int, world: int) -> List[Tuple[int, int]]:
    """Block ranges (first_block, n_blocks) per rank, bf-aligned starts, as
    even as the alignment allows.  Ranks past the end get (n0, 0)."""
    bf = block_size // 64
    n0 = -(-size // block_size)
    groups = -(-n0 // bf)                     # level-1 nodes
    out = []
    for r in range(world):
        g0 = groups * r // world
        g1 = groups * (r + 1) // world
        b0 = min(n0, g0 * bf)
        b1 = min(n0, g1 * bf)
        out.append((b0, b1 - b0))
    return out


def shard_device(N, block_size: int, salt, cid_key, d_range: int, size: int,
                 first_block: int, nb: int, d_ctext, stream) -> bytes:
    """Post blocks [first_block, first_block+nb) (bytes at device pointer
    d_range) and their level-1 nodes; returns the level-1 refs."""
    bf = block_size // 64
    m = -(-nb // bf)
    out = ctypes.create_string_buffer(64 * max(m, 1))
    N.check(N.lib.glfsx_shard_device(block_size, salt, cid_key, d_range, size,
                                     first_block, nb, d_ctext, out, stream))
    return out.raw[:64 * m]


def root_from_level1(N, block_size: int, salt, cid_key, level1: bytes, size: int):
    r = N.glfsx_root()
    N.check(N.lib.glfsx_root_from_level1(block_size, salt, cid_key, level1,
                                         len(level1) // 64, size, ctypes.byref(r)))
    return bytes(r.ref)


def write_sharded(N, dist, block_size: int, salt, cid_key, d_range: int, total: int,
                  first_block: int, nb: int, d_ctext, stream):
    """One rank's part of a sharded bigblob write, collective over
    `dist` (a torch.distributed process group; gloo carries 64 B per bf
    blocks): post this rank's blocks and level-1 nodes on its GPU, gather
    every rank's level-1 refs, and on rank 0 build levels >= 2 and the root.
    Returns (this rank's level-1 refs, the root ref on rank 0 else None).
    A blob of at most bf blocks has no level >= 2: its single level-1 node is
    posted by the rank that owns all of its blocks (rank 0)."""
    import torch
    rank, world = dist.get_rank(), dist.get_world_size()
    mine = shard_device(N, block_size, salt, cid_key, d_range, total, first_block, nb,
                        d_ctext, stream) if nb else b""
    t = torch.frombuffer(bytearray(mine), dtype=torch.uint8) if mine else \
        torch.zeros(0, dtype=torch.uint8)
    sizes = [torch.zeros(1, dtype=torch.int64) for _ in range(world)]
    dist.all_gather(sizes, torch.tensor([t.numel()], dtype=torch.int64))
    cap = max(1, int(max(x.item() for x in sizes)))
    padded = torch.zeros(cap, dtype=torch.uint8)
    padded[:t.numel()] = t
    gathered = [torch.empty(cap, dtype=torch.uint8) for _ in range(world)]
    dist.all_gather(gathered, padded)   # the only exchange: 64 B per bf blocks
    if rank != 0:
        return mine, None
    allrefs = b"".join(bytes(g[:int(k.item())].numpy().tobytes())
                       for g, k in zip(gathered, sizes))
    return mine, root_from_level1(N, block_size, salt, cid_key, allrefs, total)

"""Multi-rank sharding of one bigblob write, on CPU.

glfs_amd.shard.plan partitions the blocks into bf-aligned ranges; each rank
computes its level-1 refs (here, on CPU, with the oracle standing in for the
GPU -- test infrastructure only), the ranks all_gather them over gloo, and the
root built from the gathered refs must equal the oracle's root of the whole
blob.  The same exchange with the product on the GPU (glfs_amd.shard.
write_sharded in spawned rank processes, and bench.py's N>1 path under
torch.distributed.run) is tests/test_gpu_shard_mp.py.
"""
import os
import random

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from glfs_amd import shard


def test_plan_properties():
    rng = random.Random(1)
    for _ in range(300):
        bs = rng.choice([128, 192, 1024, 4096, 1 << 20])
        bf = bs // 64
        size = rng.randrange(0, bs * bf * rng.choice([1, 3, 9]) + 5)
        world = rng.choice([1, 2, 3, 4, 8])
        n0 = -(-size // bs)
        p = shard.plan(size, bs, world)
        assert len(p) == world
        pos = 0
        for first, nb in p:
            assert first == pos or nb == 0
            assert nb == 0 or first % bf == 0
            pos = first + nb if nb else pos
        assert sum(nb for _, nb in p) == n0


def oracle_level1(O, data, bs, first, nb, raw, idx):
    bf = bs // 64
    refs = []
    for j in range(first, first + nb):
        refs.append(O.post(raw, data[j * bs:(j + 1) * bs])[0])
    out = b""
    for k in range(0, nb, bf):
        node = b"".join(refs[k:k + bf])
        out += O.post(idx, node + bytes(bs - len(node)))[0]
    return out


def oracle_root_from_level1(O, level1, bs, idx):
    bf = bs // 64
    refs = [level1[i:i + 64] for i in range(0, len(level1), 64)]
    while len(refs) > 1:
        up = []
        for k in range(0, len(refs), bf):
            node = b"".join(refs[k:k + bf])
            up.append(O.post(idx, node + bytes(bs - len(node)))[0])
        refs = up
    return refs[0]


def _worker(rank, world, port, size, bs, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle import oracle as O
        data = O.fill_splitmix(size, 5)
        raw = O.derive_key(bytes(32), b"raw")
        idx = O.derive_key(bytes(32), b"index")
        first, nb = shard.plan(size, bs, world)[rank]
        mine = oracle_level1(O, data, bs, first, nb, raw, idx) if nb else b""
        t = torch.frombuffer(bytearray(mine), dtype=torch.uint8) if mine else \
            torch.zeros(0, dtype=torch.uint8)
        sizes = [torch.zeros(1, dtype=torch.int64) for _ in range(world)]
        dist.all_gather(sizes, torch.tensor([t.numel()], dtype=torch.int64))
        cap = max(1, int(max(s.item() for s in sizes)))
        pad = torch.zeros(cap, dtype=torch.uint8)
        pad[:t.numel()] = t
        got = [torch.empty(cap, dtype=torch.uint8) for _ in range(world)]
        dist.all_gather(got, pad)
        if rank == 0:
            level1 = b"".join(bytes(g[:int(n.item())].numpy().tobytes())
                              for g, n in zip(got, sizes))
            q.put(oracle_root_from_level1(O, level1, bs, idx))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,size", [(2, 1024 * 16 * 5 + 77), (2, 1024 * 16 * 2),
                                        (3, 1024 * 16 * 16 * 2 + 1)])
def test_gloo_shard_gather_root(O, world, size):
    bs = 1024
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + random.randrange(1000)
    ps = [ctx.Process(target=_worker, args=(r, world, port, size, bs, q)) for r in range(world)]
    [p.start() for p in ps]
    root = q.get(timeout=120)
    [p.join(60) for p in ps]
    assert all(p.exitcode == 0 for p in ps)
    want = O.create(O.fill_splitmix(size, 5), bs, salt=None, closed_form=True)[0]
    assert root == want

"""The product's multi-GPU write path across processes (SURVEY 8e,
bigblob/blob.go:165-206 split by block ranges), rehearsed on one GPU.

Each rank is a fresh child process (multiprocessing "spawn"; the test process
is never exec'd) that fills its bf-aligned block range of a synthetic blob
in HBM and runs glfs_amd.shard.write_sharded -- glfsx_shard_device, a gloo
all_gather of the level-1 refs, glfsx_root_from_level1 on rank 0 -- the same
function bench.py's N>1 step runs.  The root must equal the N=1
glfsx_create_device root over the whole blob, and every rank's level-1 refs
the oracle's.  bench.py itself is then run under torch.distributed.run with
2 ranks and must print that root.
"""
import ctypes
import json
import os
import random
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MIB, GIB = 1 << 20, 1 << 30


def _worker(rank, world, port, total, bs, seed, q, dev=0):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist
    from glfs_amd import _native as N, shard
    try:
        torch.cuda.set_device(dev)
        N.set_device(dev)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        first, nb = shard.plan(total, bs, world)[rank]
        n = min(nb * bs, total - first * bs)
        data = torch.empty(max(n, 1), dtype=torch.uint8, device="cuda")
        N.check(N.lib.glfsx_fill_splitmix_device(data.data_ptr(), first * bs, n, seed, None))
        torch.cuda.synchronize()
        mine, root = shard.write_sharded(N, dist, bs, None, None, data.data_ptr(), total,
                                         first, nb, None, None)
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, first, nb, mine, root, None))
    except Exception as e:  # reported to the parent
        q.put((rank, 0, 0, b"", None, repr(e)))


def _run_ranks(world, total, bs, seed, per_rank_device=False):
    """world ranks as spawned children; rank r on device r when
    per_rank_device (distinct GPUs), else all on device 0 (rehearsal)."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + random.randrange(2000)
    ps = [ctx.Process(target=_worker, args=(r, world, port, total, bs, seed, q,
                                            r if per_rank_device else 0))
          for r in range(world)]
    [p.start() for p in ps]
    out = {}
    for _ in range(world):
        rank, first, nb, mine, root, err = q.get(timeout=240)
        assert err is None, (rank, err)
        out[rank] = (first, nb, mine, root)
    [p.join(60) for p in ps]
    assert all(p.exitcode == 0 for p in ps)
    return out


def _whole_root(total, bs, seed):
    import torch
    from glfs_amd import _native as N
    t = torch.empty(total, dtype=torch.uint8, device="cuda")
    N.check(N.lib.glfsx_fill_splitmix_device(t.data_ptr(), 0, total, seed, None))
    r = N.glfsx_root()
    N.check(N.lib.glfsx_create_device(bs, None, None, t.data_ptr(), total, None,
                                      ctypes.byref(r), None, None))
    torch.cuda.synchronize()
    return bytes(r.ref), t


def _oracle_level1(O, t, bs, first, nb):
    """Level-1 refs of blocks [first, first+nb): threaded oracle over the
    bytes copied down from HBM, 1 GiB at a time."""
    import numpy as np
    L = O.lib()
    raw, idx = O.derive_key(bytes(32), b"raw"), O.derive_key(bytes(32), b"index")
    bf = bs // 64
    total = t.numel()
    refs = b""
    step = max(1, GIB // bs)
    for b0 in range(first, first + nb, step):
        k = min(step, first + nb - b0)
        lo, hi = b0 * bs, min((b0 + k) * bs, total)
        pt = t[lo:hi].cpu().numpy()
        out = np.empty(64 * k, dtype=np.uint8)
        L.oracle_post_batch(out.ctypes.data, None, raw, pt.ctypes.data, hi - lo, bs, None, 16)
        refs += out.tobytes()
    return b"".join(O.post(idx, refs[i:i + 64 * bf].ljust(bs, b"\0"))[0]
                    for i in range(0, len(refs), 64 * bf))


@pytest.mark.parametrize("world,bs,nblocks", [
    (2, MIB, 2 * 16384),             # 2 x 16 GiB at 1 MiB blocks: 1 level-1 node each
    (3, 64 << 10, 1024 * 3 + 5),     # 4 level-1 nodes over 3 ranks, ragged last
])
def test_sharded_write_across_processes(gpu, O, world, bs, nblocks):
    total = nblocks * bs - (777 if bs < MIB else 0)
    seed = 3
    got = _run_ranks(world, total, bs, seed)
    want_root, t = _whole_root(total, bs, seed)
    assert got[0][3] == want_root
    assert sum(nb for _, nb, _, _ in got.values()) == -(-total // bs)
    for rank, (first, nb, mine, _) in got.items():
        if nb:
            assert mine == _oracle_level1(O, t, bs, first, nb), rank
    if world == 2 and bs == MIB:
        # bench.py's own N=2 path (torch.distributed.run, 2 ranks; on one
        # GPU a rehearsal) must print the same root for the same 32 GiB
        # blob (seed 3)
        import torch
        env = dict(os.environ)
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
               "--nproc-per-node", "2", "--master-addr", "127.0.0.1",
               "--master-port", str(31000 + random.randrange(2000)),
               os.path.join(ROOT, "bench.py"), "--gpus", "2", "--size-gib", "16",
               "--steps", "1", "--warmup", "0", "--no-extras"]
        if torch.cuda.device_count() < 2:
            cmd.append("--rehearse")
        p = subprocess.run(cmd, capture_output=True, text=True, timeout=400, env=env, cwd=ROOT)
        assert p.returncode == 0, p.stderr[-3000:]
        line = [ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1]
        rec = json.loads(line)
        assert rec["n_gpus"] == 2 and rec["root_cid"] == want_root[:32].hex()


@pytest.mark.parametrize("gpus", [2, 8])
def test_bench_one_process_gpus(gpu, gpus):
    """bench.py --gpus N without a launcher drives N devices from ONE
    process (glfsx_create_devices).  With fewer GPUs visible it must refuse
    (exit 2) unless --rehearse, which names device 0 N times and must print
    n_gpus N, rehearsal true and the N = 1 root of the same N x 16 GiB blob
    (parts = the splitmix stream at offsets k x 16 GiB, seed 3).  N = 8 is
    BASELINE config 5's level structure (8 level-1 nodes under one root)
    at 16 GiB per part, ctext off so the 128 GiB fit one GPU's HBM."""
    import torch
    total = gpus * 16 * GIB
    want_root, t = _whole_root(total, MIB, 3)
    del t
    torch.cuda.empty_cache()
    base = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(gpus), "--size-gib",
            "16", "--steps", "1", "--warmup", "0", "--no-extras"]
    if gpus > 2:
        base.append("--no-ctext")
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    rehearsal = torch.cuda.device_count() < gpus
    if rehearsal:
        p = subprocess.run(base, capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
        assert p.returncode == 2 and "GPU(s) visible" in p.stderr, (p.returncode,
                                                                    p.stderr[-2000:])
        base.append("--rehearse")
    p = subprocess.run(base, capture_output=True, text=True, timeout=400, env=env, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-3000:]
    rec = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1])
    assert rec["n_gpus"] == gpus and rec["root_cid"] == want_root[:32].hex()
    assert rec["rehearsal"] is rehearsal
    assert rec["config"]["blob_bytes"] == total
    assert rec["config"]["posts_per_step"] == total // MIB + gpus + 1
    assert len(rec["per_device_ms"]["parts"]) == gpus

"""bench.py -- bigblob write path, device-resident, GiB/s hashed.

Workload (BASELINE.json metric, configs[2] / configs[4]): a synthetic blob of
--size-gib GiB per GPU (default 64) at 1 MiB blocks, resident in HBM before
the timed region.  One step = the whole bigblob write of that blob on the GPU
(bigblob/blob.go:85-206 closed form): every data block posted (DEK = keyed
BLAKE3, ChaCha20 ctext written to HBM, CID = BLAKE3 of ctext), the index
nodes above them, and the root.  With N GPUs each rank owns a contiguous,
bf-aligned block range of an N x size blob (weak scaling, no data-path
collective); the level-1 refs (64 B per 16 GiB) are gathered once per step
and rank 0 builds the root.

Prints ONE JSON line (rank 0).  Extra objects: roofline (dominant kernel,
HIP events on the launch stream), cpu_baseline (the oracle on host cores),
host_round_trip (host memory -> GPU -> host ctext + refs), valu (second
roofline).  Data is synthetic: a splitmix64 byte stream generated on the GPU
(glfsx_fill_splitmix_device).  Only the cpu_baseline leg touches oracle/.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

GIB, MIB = 1 << 30, 1 << 20
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: 8.0 TB/s spec
# int-VALU roofline (DESIGN.md "Rooflines").  gfx950 issues wave64 integer
# ops in two classes (tools/mix.hip): full rate, 2 cycles (v_add_u32,
# v_xor_b32, v_lshrrev_b32, v_bitop3_b32, VGPR/literal operands) and half
# rate, 4 cycles (v_add3_u32, v_alignbit_b32, v_perm_b32, v_lshlrev_b32, any
# SGPR operand).  The ideal time of a kernel is its algorithmic instruction
# mix at those costs on 1024 SIMDs at the 2.4 GHz peak clock:
#   BLAKE3 G  = 6 full (2 add, 4 xor) + 6 half (2 add3, 4 alignbit) = 36 cyc
#   ChaCha QR = 8 full (4 add, 4 xor) + 4 half (4 alignbit)          = 32 cyc
#   compression = 56 G + 8 xor; one parent per 16 blocks (1 MiB, G = 4)
#   ChaCha block = 80 QR - 3 uniform QRs (hoisted) + 16 xor + 5 full adds
#                  + 8 half adds (SGPR key words)
SIMDS, PEAK_GHZ = 1024, 2.4
_COMPRESS = 56 * 36 + 8 * 2
_CHACHA = (80 - 3) * 32 + 16 * 2 + 5 * 2 + 8 * 4
IDEAL_CYCLES_PER_BLOCK = {"dek": _COMPRESS * (1 + 1 / 16),
                          "cid": _CHACHA + _COMPRESS * (1 + 1 / 16)}
# VALU lane-instructions per plaintext byte, measured with rocprofv3
# SQ_INSTS_VALU x 64 / bytes (profiles/r1/summary.json).
INSTR_PER_BYTE = {"dek": 11.60, "cid": 26.53}


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--size-gib", type=float, default=64.0, help="blob bytes per GPU")
    p.add_argument("--block-size", type=int, default=MIB)
    p.add_argument("--seed", type=int, default=3)
    p.add_argument("--no-ctext", action="store_true",
                   help="do not write ctext (NOT the headline configuration)")
    p.add_argument("--no-extras", action="store_true",
                   help="skip roofline/cpu/host legs (profiling runs)")
    p.add_argument("--cpu-sample-mib", type=int, default=3072)
    p.add_argument("--host-rt-gib", type=float, default=4.0)
    p.add_argument("--rehearse", action="store_true",
                   help="allow fewer visible GPUs than --gpus: parts / ranks share "
                        "devices round-robin (a rehearsal on one box, not a measurement)")
    return p.parse_args(argv)


def plan_devices(gpus: int, world: int, local: int, ndev: int, rehearse: bool):
    """Which GPUs this process drives (one part of the blob each).

    * world > 1 -- launched by torch.distributed.run, one rank per GPU: rank
      `local` drives device `local`; --gpus must equal the world size.
    * world == 1, gpus > 1 -- ONE process drives `gpus` devices through
      glfsx_create_devices (the shape of a Go process on the node calling the
      C-ABI).
    * world == 1, gpus == 1 -- the headline, device 0.
    Fewer visible devices than needed is an error unless `rehearse` (then
    devices are named round-robin).  Returns (mode, devices); raises
    ValueError with the reason."""
    if gpus < 1:
        raise ValueError(f"--gpus {gpus}: need at least 1")
    if ndev < 1:
        raise ValueError("no GPU visible (the glfsx path has no CPU fallback)")
    if world > 1:
        if gpus != world:
            raise ValueError(f"--gpus {gpus} under a launcher with WORLD_SIZE {world}: "
                             "one rank per GPU, they must match")
        if local >= ndev and not rehearse:
            raise ValueError(f"rank {local} needs device {local} but only {ndev} visible "
                             "(--rehearse shares devices)")
        return "ranks", [local % ndev]
    if gpus > ndev and not rehearse:
        raise ValueError(f"--gpus {gpus} but only {ndev} GPU(s) visible "
                         "(--rehearse shares devices round-robin)")
    return ("one_process" if gpus > 1 else "single"), [k % ndev for k in range(gpus)]


def main():
    args = parse()
    import torch
    import torch.distributed as dist
    from glfs_amd import _native as N

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    ndev = torch.cuda.device_count()   # counts without initialising the GPU
    try:
        mode, devs = plan_devices(args.gpus, world, local, ndev, args.rehearse)
    except ValueError as e:
        print(f"bench.py: {e}", file=sys.stderr, flush=True)
        sys.exit(2)
    # host buffers, the tmpfs file and the library's copy threads on the
    # GPU's NUMA node (file feed 27-29 -> 35-39 GiB/s on a two-socket box;
    # DESIGN.md section 8); a one-process run over GPUs on both sockets
    # stays unbound
    nodes = {gpu_numa_node(torch, d) for d in devs}
    host_node = numa_bind(torch, devs[0]) if len(nodes) == 1 else None
    if mode == "one_process":
        return main_one_process(args, devs, host_node)
    dev = devs[0]
    torch.cuda.set_device(dev)
    N.set_device(dev)
    if world > 1:
        # gloo carries only the 256-B level-1 gather, the barriers and the
        # max-over-ranks time: no collective on the data path.
        dist.init_process_group(os.environ.get("GLFS_DIST_BACKEND", "gloo"))

    from glfs_amd import shard
    bs = args.block_size
    bf = bs // 64
    per_req = int(args.size_gib * GIB) // bs * bs   # bytes per rank, whole blocks
    if world > 1:
        per_req = max(bf, per_req // bs // bf * bf) * bs   # bf-aligned shards
    total = per_req * world
    n0 = total // bs
    first, nb = shard.plan(total, bs, world)[rank]
    per = nb * bs

    stream = torch.cuda.Stream()
    sp = ctypes.c_void_p(stream.cuda_stream)
    with torch.cuda.stream(stream):
        data = torch.empty(per, dtype=torch.uint8, device="cuda")
        ctext = None if args.no_ctext else torch.empty(per, dtype=torch.uint8, device="cuda")
        N.check(N.lib.glfsx_fill_splitmix_device(data.data_ptr(), first * bs, per,
                                                  args.seed, sp))
    stream.synchronize()
    ct_ptr = None if ctext is None else ctext.data_ptr()

    root = N.glfsx_root()
    n_posts = ctypes.c_uint64()
    root_ref = [b""]

    def step():
        if world == 1:
            N.check(N.lib.glfsx_create_device(bs, None, None, data.data_ptr(), per, ct_ptr,
                                              ctypes.byref(root), ctypes.byref(n_posts), sp))
            root_ref[0] = bytes(root.ref)
            return
        _, r = shard.write_sharded(N, dist, bs, None, None, data.data_ptr(), total, first, nb,
                                   ct_ptr, sp)
        if rank == 0:
            root_ref[0] = r

    def barrier():
        if world > 1:
            dist.barrier()

    for _ in range(args.warmup):
        step()
    barrier()
    torch.cuda.synchronize()
    N.check(N.lib.glfsx_clock_probe(1, None))   # (synchronous; before the clock starts)
    reruns0 = N.lib.glfsx_fused_failures()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    barrier()
    dt = time.perf_counter() - t0
    reruns = {"headline": N.lib.glfsx_fused_failures() - reruns0}
    probe = (ctypes.c_uint64 * 2)()
    N.check(N.lib.glfsx_clock_probe(0, probe))
    step_clock = round(probe[0] / probe[1] * 0.1, 3) if probe[1] else None
    if world > 1:
        tt = torch.tensor([dt], dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
    ms = dt / args.steps * 1e3
    gibs = total / GIB * args.steps / dt

    out = {
        "metric": "GiB/s hashed, device-resident 1 MiB chunks, bigblob write; 1/2/4/8 MI355X",
        "value": round(gibs, 2),
        "unit": "GiB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u32",
        "data": "synthetic (splitmix64 byte stream, generated in HBM)",
        "config": {"workload": f"bigblob write {per / GIB:g} GiB/GPU @ {bs // 1024} KiB "
                               f"blocks, device-resident, ctext {'off' if ctext is None else 'to HBM'}",
                   "blob_bytes": total, "block_size": bs, "blocks": n0,
                   "posts_per_step": n_posts.value if world == 1 else None,
                   "parallelism": f"disjoint block ranges x{world}"},
        "root_cid": root_ref[0][:32].hex() if rank == 0 else None,
        "host_numa_node": host_node,
        "held_clock_GHz": step_clock,
        "held_clock_what": "shader clock over the timed steps' hashing launches on this "
                           "rank's GPU (s_memtime cycles / s_memrealtime ticks summed over "
                           "every k_pass workgroup, glfsx_clock_probe); peak 2.4",
    }

    if not args.no_extras:
        if rank == 0:
            out["roofline"], out["valu"] = roofline(torch, N, data, ctext, per, bs, stream, sp,
                                                    step_ms=ms, total_bytes=per)
        del ctext
        # host round trip on every rank at once (N PCIe links, N host feeders):
        # aggregate bytes over the slowest rank's time
        def slowest(sec):
            """barrier-aligned rep: the slowest rank's time"""
            if world == 1:
                return sec
            tt = torch.tensor([sec], dtype=torch.float64)
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            return float(tt.item())

        hrt = host_round_trip(N, args, bs, barrier, slowest)
        if rank == 0 and world == 1 and args.host_rt_gib > 0:
            out["concat"] = concat_leg(N)
            out["postblob_latency"] = postblob_latency(N)
            out["postblob_concurrency"] = postblob_concurrency(N)
        if hrt is not None and world > 1:
            hrt["value"] = round(world * hrt["value"], 2)
            hrt["bytes"] *= world
            if "sinks" in hrt:   # aggregates too, like value
                hrt["sinks"] = {k: round(world * v, 2) for k, v in hrt["sinks"].items()}
            hrt["what"] += f"; {world} ranks at once, aggregate over the slowest rank"
        if world > 1:
            # SURVEY 8e in ONE process (the C-ABI a Go caller on this node
            # would use): rank 0 drives every GPU while the others wait
            barrier()
            if rank == 0:
                try:
                    out["one_process_multi_gpu"] = one_process_multi_gpu(torch, N, args, world,
                                                                         bs, dev)
                except Exception as e:  # reported, never fatal to the bench line
                    out["one_process_multi_gpu"] = {"error": repr(e)[:500]}
            barrier()
        if rank == 0:
            out["host_round_trip"] = hrt
            if world == 1:   # the CPU baseline is an N=1 figure (rank 0 only)
                out["cpu_baseline"] = cpu_baseline(args)
            if args.host_rt_gib > 0:
                r0 = N.lib.glfsx_fused_failures()
                out["config2"] = config2_leg(torch, N, stream, sp)
                reruns["config2"] = N.lib.glfsx_fused_failures() - r0
                out["small_blobs"] = small_blobs(torch, N, stream, sp)
                out["small_blobs_from_host"] = small_blobs_from_host(torch, N, stream, sp)
                r0 = N.lib.glfsx_fused_failures()
                out["config4_end_to_end"] = config4_end_to_end(torch, N, stream, sp)
                reruns["config4"] = N.lib.glfsx_fused_failures() - r0
                if world == 1 and "cpu_baseline" in out:
                    out["cpu_baseline"].update(
                        cpu_baseline_configs(args, out["config2"]["root_cid"]))
    # a one-launch split post that failed was discarded and re-run with two
    # launches inside the timed region: the line says how often (0 expected),
    # and a non-zero count fails the run (glfsx_fused_failures)
    out["fused_reruns"] = reruns
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()
    if any(reruns.values()):
        print(f"bench.py: one-launch split posts were re-run: {reruns}", file=sys.stderr,
              flush=True)
        sys.exit(3)


def gpu_numa_node(torch, dev):
    """The NUMA node of GPU `dev` (sysfs of its PCI function), or None."""
    try:
        p = torch.cuda.get_device_properties(dev)
        bdf = f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}.0"
        with open(f"/sys/bus/pci/devices/{bdf}/numa_node") as f:
            node = int(f.read())
        return node if node >= 0 else None
    except (OSError, ValueError, AttributeError):
        return None


def numa_bind(torch, dev):
    """Run this process (and the threads it starts later, e.g. the
    library's copy pool) on the CPUs of GPU dev's NUMA node, so host buffers
    are first touched there; returns the node, or None if unknown."""
    node = gpu_numa_node(torch, dev)
    if node is None:
        return None
    try:
        with open(f"/sys/devices/system/node/node{node}/cpulist") as f:
            cpus = set()
            for part in f.read().strip().split(","):
                lo, _, hi = part.partition("-")
                cpus.update(range(int(lo), int(hi or lo) + 1))
        allowed = os.sched_getaffinity(0) & cpus
        if not allowed:
            return None
        os.sched_setaffinity(0, allowed)
        return node
    except (OSError, ValueError):
        return None


def main_one_process(args, devs, host_node=None):
    """N GPUs from ONE process (BASELINE config 5's shape, the way
    a Go process on the node drives them through the C-ABI): the blob is N
    parts of --size-gib GiB, part k resident in HBM on devs[k] (bytes = the
    splitmix stream at offset k x part, so the blob is the N = 1 stream over
    N x part bytes), ctext written beside it.  One step = one
    glfsx_create_devices call: every device posts its part's data blocks and
    level-1 nodes at once (a worker thread per device, no collective), the
    level-1 refs are gathered on the host and the levels above posted on
    devs[0].  ms_per_step = the call's wall time (it returns when every part
    and the root are done); per-device GPU times from HIP events on each
    part's stream (glfsx_create_devices_ms)."""
    import torch
    from glfs_amd import _native as N
    bs = args.block_size
    bf = bs // 64
    span = bs * bf                              # one level-1 node: 16 GiB at 1 MiB
    per = max(span, int(args.size_gib * GIB) // span * span)
    nd = len(devs)
    total = per * nd
    bufs, cts = [], []
    for k, d in enumerate(devs):
        torch.cuda.set_device(d)
        N.set_device(d)
        t = torch.empty(per, dtype=torch.uint8, device=f"cuda:{d}")
        c = None if args.no_ctext else torch.empty(per, dtype=torch.uint8, device=f"cuda:{d}")
        N.check(N.lib.glfsx_fill_splitmix_device(t.data_ptr(), k * per, per, args.seed, None))
        bufs.append(t)
        cts.append(c)
    for d in sorted(set(devs)):
        torch.cuda.synchronize(d)
    home = devs[0]
    torch.cuda.set_device(home)
    N.set_device(home)
    cdevs = (ctypes.c_int * nd)(*devs)
    ptrs = (ctypes.c_void_p * nd)(*[t.data_ptr() for t in bufs])
    sizes = (ctypes.c_uint64 * nd)(*([per] * nd))
    cptrs = None if args.no_ctext else (ctypes.c_void_p * nd)(*[c.data_ptr() for c in cts])
    root, posts = N.glfsx_root(), ctypes.c_uint64()
    msb = (ctypes.c_float * (nd + 1))()

    def step():
        N.check(N.lib.glfsx_create_devices(bs, None, None, nd, cdevs, ptrs, sizes, cptrs, None,
                                           ctypes.byref(root), ctypes.byref(posts)))
        k = N.lib.glfsx_create_devices_ms(msb, nd + 1)
        return list(msb[:max(0, min(k, nd + 1))])

    def sync_all():
        for d in sorted(set(devs)):
            torch.cuda.synchronize(d)

    for _ in range(args.warmup):
        step()
    sync_all()
    reruns0 = N.lib.glfsx_fused_failures()
    t0 = time.perf_counter()
    parts = [step() for _ in range(args.steps)]
    sync_all()
    dt = time.perf_counter() - t0
    reruns = {"headline": N.lib.glfsx_fused_failures() - reruns0}
    ms = dt / args.steps * 1e3
    mean = [sum(p[k] for p in parts) / len(parts) for k in range(len(parts[0]))] if parts else []
    out = {
        "metric": "GiB/s hashed, device-resident 1 MiB chunks, bigblob write; 1/2/4/8 MI355X",
        "value": round(total / GIB * args.steps / dt, 2),
        "unit": "GiB/s",
        "n_gpus": nd,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u32",
        "data": "synthetic (splitmix64 byte stream, generated in HBM on each GPU)",
        "config": {"workload": f"bigblob write {per / GIB:g} GiB/GPU @ {bs // 1024} KiB "
                               f"blocks, device-resident, ctext "
                               f"{'off' if args.no_ctext else 'to HBM'}",
                   "blob_bytes": total, "block_size": bs, "blocks": total // bs,
                   "posts_per_step": posts.value,
                   "parallelism": f"disjoint block ranges x{nd}, one process "
                                  "(glfsx_create_devices)"},
        "devices": devs,
        "rehearsal": len(set(devs)) < nd,
        "host_numa_node": host_node,
        "root_cid": bytes(root.ref)[:32].hex(),
        "per_device_ms": {"parts": [round(x, 3) for x in mean[:nd]],
                          "levels_above": round(mean[nd], 3) if len(mean) > nd else None,
                          "what": "mean GPU ms per step: each part's data blocks + level-1 "
                                  "nodes on its device, then the levels >= 2 on devs[0] (HIP "
                                  "events on the stream that ran them)"},
    }
    if not args.no_extras:
        stream = torch.cuda.Stream(device=home)
        sp = ctypes.c_void_p(stream.cuda_stream)
        out["roofline"], out["valu"] = roofline(torch, N, bufs[0], cts[0], per, bs, stream, sp,
                                                step_ms=ms, total_bytes=per)
        out["roofline"]["device"] = home
        del bufs, cts
        if args.host_rt_gib > 0:
            out["host_round_trip"] = multi_lane_host(torch, N, args, devs, bs)
    out["fused_reruns"] = reruns
    print(json.dumps(out), flush=True)
    if any(reruns.values()):
        print(f"bench.py: one-launch split posts were re-run: {reruns}", file=sys.stderr,
              flush=True)
        sys.exit(3)


def multi_lane_host(torch, N, args, devs, bs):
    """One host stream over every GPU: one Writer (pre-hashed store) with its
    batches round-robin over the devices' lanes (glfsx_writer_set_devices),
    fed (a) from pageable memory in 64 MiB writes and (b) from a tmpfs file
    by the parallel pread feeder (glfsx_writer_read_fd).  PCIe-inclusive,
    never the headline value."""
    import numpy as np
    nd = len(devs)
    # 4 GiB per GPU up to 16 GiB in all (the legs stay within a minute at N = 8)
    n = int(min(args.host_rt_gib * nd, 4.0 * nd, 16.0) * GIB) // bs * bs
    host = host_stream(torch, N, n, args.seed)
    store_post = ctypes.cast(N.lib.glfsx_store_post, N.POST_FN)
    root = N.glfsx_root()
    best = {}
    for label, lanes in (("one_gpu", devs[:1]), ("all_gpus", devs)):
        for _ in range(3):
            st = N.lib.glfsx_store_new(bs, N.GLFSX_STORE_TRUST, 0, 0, None)
            err = ctypes.c_int()
            t = time.perf_counter()
            w = N.lib.glfsx_writer_new(bs, bs, None, None, store_post, st, ctypes.byref(err))
            assert w, N.last_error()
            rc = N.lib.glfsx_writer_set_devices(w, (ctypes.c_int * len(lanes))(*lanes),
                                                len(lanes))
            if rc == 0:
                rc = N.lib.glfsx_writer_copy(w, host.ctypes.data, n, 64 * MIB)
            if rc == 0:
                rc = N.lib.glfsx_writer_finish(w, ctypes.byref(root))
            msg = (N.lib.glfsx_writer_error(w) or b"").decode()
            N.lib.glfsx_writer_free(w)
            dt = time.perf_counter() - t
            N.lib.glfsx_store_free(st)
            N.check(rc, msg)
            best[label] = min(best.get(label, dt), dt)
    want = bytes(root.ref)
    res = {"value": round(n / GIB / best["all_gpus"], 2), "unit": "GiB/s",
           "one_gpu_value": round(n / GIB / best["one_gpu"], 2), "bytes": n,
           "root_cid": want[:32].hex(),
           "what": f"one Writer, one pageable host stream of {n / GIB:g} GiB in 64 MiB "
                   f"writes, batches round-robin over {nd} GPUs (glfsx_writer_set_devices), "
                   "pre-hashed store; one_gpu_value: the same on the first GPU only; best "
                   "of 3"}
    res["file_feed"] = file_feed(N, host, bs, {"lanes_all": list(devs)}, want)
    del host
    return res


def host_stream(torch, N, n, seed):
    """n bytes of the splitmix stream in pageable host memory (generated on
    the GPU, copied down)."""
    import numpy as np
    host = np.empty(n, dtype=np.uint8)
    dev = torch.empty(64 * MIB, dtype=torch.uint8, device="cuda")
    for off in range(0, n, 64 * MIB):
        m = min(64 * MIB, n - off)
        N.check(N.lib.glfsx_fill_splitmix_device(dev.data_ptr(), off, m, seed, None))
        torch.cuda.synchronize()
        host[off:off + m] = dev[:m].cpu().numpy()
    del dev
    return host


def file_feed(N, host, bs, lane_sets, want_ref, reps=3):
    """bigblob.Create fed by a file (glfs.go:53 io.Copy from an *os.File;
    blob.go:209-217): the bytes of `host` written to a tmpfs file, then read
    by glfsx_writer_read_fd -- several threads pread each batch straight into
    the Writer's pinned staging while earlier batches upload, hash and
    download -- into a pre-hashed store, for each lane set.  The root must
    equal want_ref (the same bytes through glfsx_create).  Best of reps; the
    file is removed afterwards."""
    import tempfile
    n = host.size
    d = "/dev/shm" if os.path.isdir("/dev/shm") else tempfile.gettempdir()
    fd_w, path = tempfile.mkstemp(prefix="glfsx_feed_", dir=d)
    res = {}
    try:
        with os.fdopen(fd_w, "wb") as f:
            for off in range(0, n, 256 * MIB):
                f.write(memoryview(host[off:off + 256 * MIB]))
        store_post = ctypes.cast(N.lib.glfsx_store_post, N.POST_FN)
        root, got = N.glfsx_root(), ctypes.c_uint64()
        fd = os.open(path, os.O_RDONLY)
        try:
            for label, lanes in lane_sets.items():
                best = None
                for _ in range(reps):
                    st = N.lib.glfsx_store_new(bs, N.GLFSX_STORE_TRUST, 0, 0, None)
                    err = ctypes.c_int()
                    t = time.perf_counter()
                    w = N.lib.glfsx_writer_new(bs, bs, None, None, store_post, st,
                                               ctypes.byref(err))
                    assert w, N.last_error()
                    rc = 0
                    if len(lanes) > 1:
                        rc = N.lib.glfsx_writer_set_devices(
                            w, (ctypes.c_int * len(lanes))(*lanes), len(lanes))
                    if rc == 0:
                        rc = N.lib.glfsx_writer_read_fd(w, fd, 0, n, ctypes.byref(got))
                    if rc == 0:
                        rc = N.lib.glfsx_writer_finish(w, ctypes.byref(root))
                    msg = (N.lib.glfsx_writer_error(w) or b"").decode()
                    N.lib.glfsx_writer_free(w)
                    dt = time.perf_counter() - t
                    N.lib.glfsx_store_free(st)
                    N.check(rc, msg)
                    assert got.value == n and bytes(root.ref) == want_ref, "file feed root"
                    best = dt if best is None else min(best, dt)
                res[label] = round(n / GIB / best, 2)
        finally:
            os.close(fd)
    finally:
        os.unlink(path)
    res["what"] = (f"bigblob.Create from a {n / GIB:g} GiB tmpfs file ({d}): "
                   "glfsx_writer_read_fd, each 64 MiB batch pread by up to 16 threads straight "
                   "into the pinned staging, pre-hashed store; root equal to glfsx_create's of "
                   "the same bytes; best of 3")
    return res


def roofline(torch, N, data, ctext, per, bs, stream, sp, reps=5, step_ms=None, total_bytes=None):
    """Per-kernel average duration with HIP events on the launch stream: the
    DEK pass (reads ptext) and the ChaCha20+CID pass (reads ptext, writes
    ctext).  achieved = algorithmic bytes per launch / avg duration."""
    nblk = per // bs
    refs = torch.zeros(64 * nblk, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    salt = bytes(32)
    ct = None if ctext is None else ctext.data_ptr()
    times = {"dek": [], "cid": []}
    # the clock the chip held over these very launches: every k_pass
    # workgroup adds its lifetime in shader-clock cycles and in 100 MHz ticks
    # to two device counters (glfsx_clock_probe), read after each timed pass
    probe = (ctypes.c_uint64 * 2)()
    clk = {"dek": [0, 0], "cid": [0, 0]}
    N.check(N.lib.glfsx_clock_probe(1, None))
    with torch.cuda.stream(stream):
        for rep in range(reps + 1):
            e = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
            e[0].record(stream)
            N.check(N.lib.glfsx_dek_batch_device(salt, data.data_ptr(), per, bs,
                                                 refs.data_ptr(), sp))
            e[1].record(stream)
            e[1].synchronize()
            N.check(N.lib.glfsx_clock_probe(1, probe))
            if rep:   # the first rep is the warm-up
                clk["dek"] = [clk["dek"][0] + probe[0], clk["dek"][1] + probe[1]]
            e[2].record(stream)
            N.check(N.lib.glfsx_cid_batch_device(data.data_ptr(), per, bs, ct,
                                                 refs.data_ptr(), None, sp))
            e[3].record(stream)
            e[3].synchronize()
            N.check(N.lib.glfsx_clock_probe(1, probe))
            if rep:
                clk["cid"] = [clk["cid"][0] + probe[0], clk["cid"][1] + probe[1]]
            times["dek"].append(e[0].elapsed_time(e[1]))
            times["cid"].append(e[2].elapsed_time(e[3]))
    avg = {k: sum(v[1:]) / reps for k, v in times.items()}  # first rep = warm-up
    clock = {k: v[0] / v[1] * 0.1 for k, v in clk.items() if v[1]}   # GHz
    read = None
    if ct is not None:
        # read side (getF decrypt, ref.go:113-126): ctext -> ptext written over
        # the plaintext buffer (identical bytes), DEKs from the refs above
        tr = []
        with torch.cuda.stream(stream):
            for _ in range(reps + 1):
                e = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
                e[0].record(stream)
                N.check(N.lib.glfsx_decrypt_batch_device(ct, per, bs, refs.data_ptr(),
                                                         data.data_ptr(), sp))
                e[1].record(stream)
                e[1].synchronize()
                tr.append(e[0].elapsed_time(e[1]))
        rms = sum(tr[1:]) / reps
        read = {"value": round(per / GIB / (rms * 1e-3), 1), "unit": "GiB/s", "ms": round(rms, 3),
                "what": "batched getF decrypt (ChaCha20 with each block's DEK), HBM->HBM"}
    # algorithmic bytes = 1 B of HBM read per plaintext byte
    # hashed; a launch of either pass covers `per` plaintext bytes.  The CID
    # pass also writes the ctext (1 B/B more): that is in `traffic` (PMC) and
    # kernel_traffic_frac, not in `achieved`.
    alg = {"dek": per, "cid": per}
    kern_bytes = {"dek": per, "cid": per * (2 if ct is not None else 1)}
    dom = max(avg, key=avg.get)
    achieved = alg[dom] / (avg[dom] * 1e-3) / 1e9
    traffic = None
    tf = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if os.path.exists(tf):
        try:
            pm = json.load(open(tf))
            t = pm.get(dom, {})
            # profiled at the 64 GiB launch; traffic is linear in blocks
            traffic = int(t["hbm_bytes_per_launch"] * kern_bytes[dom] / t["algorithmic_bytes"])
        except Exception:
            traffic = None
    ms_step = step_ms if step_ms else None
    roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
            "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
            "kernel": {"dek": "k_pass<4,false,true,2> (keyed BLAKE3, DEK)",
                       "cid": "k_pass<4,true,true,1> (ChaCha20 + ctext store + BLAKE3 CID)"}[dom],
            "algorithmic_bytes_per_launch": alg[dom],
            "algorithmic_model": "SURVEY 8(d): 1 B of HBM read per plaintext byte hashed",
            "kernel_traffic_frac": (round(traffic / (avg[dom] * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
                                    if traffic else None),
            "step_frac": (round(total_bytes / (ms_step * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
                          if ms_step else None),
            "avg_ms": {k: round(v, 4) for k, v in avg.items()},
            "hashed_GBps": {k: round(per / (v * 1e-3) / 1e9, 1) for k, v in avg.items()}}
    # ideal: each wave-cycle of a SIMD covers 64 lanes x 64 B blocks
    ideal_ms = {k: IDEAL_CYCLES_PER_BLOCK[k] * (per / 4096) / (SIMDS * PEAK_GHZ * 1e9) * 1e3
                for k in avg}
    valu = {"bound": "valu", "unit": "ms per launch",
            "model": "class-weighted issue: full-rate ops 2 cyc, half-rate 4 cyc per wave64 "
                     "instruction, 1024 SIMDs at 2.4 GHz (DESIGN.md Rooflines)",
            "ideal_cycles_per_64B_block": {k: round(v, 1) for k, v in IDEAL_CYCLES_PER_BLOCK.items()},
            "ideal_ms": {k: round(v, 3) for k, v in ideal_ms.items()},
            "achieved_ms": {k: round(v, 3) for k, v in avg.items()},
            "frac": {k: round(ideal_ms[k] / avg[k], 3) for k in avg},
            "held_clock_GHz": {k: round(v, 3) for k, v in clock.items()},
            "frac_at_held_clock": {k: round(ideal_ms[k] * PEAK_GHZ / clock[k] / avg[k], 3)
                                   for k in avg if k in clock},
            "held_clock_source": "this run: the timed launches themselves (every k_pass "
                                 "workgroup sums its lifetime in s_memtime shader-clock "
                                 "cycles and s_memrealtime 100 MHz ticks, glfsx_clock_probe; "
                                 "GHz = cycles / ticks x 0.1), same reps as achieved_ms",
            "instr_per_byte": INSTR_PER_BYTE}
    del refs
    roof["read_side"] = read
    return roof, valu


def job_cores():
    """Threads the CPU baselines run: the job's core share (OMP_NUM_THREADS,
    16 on the GPU box), at most the CPUs this process may run on."""
    aff = len(os.sched_getaffinity(0))
    return max(1, min(int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or aff, aff))


def core_info():
    """What the job_cores figures ran on: the thread
    count used, the affinity mask's size, OMP_NUM_THREADS and the host's
    whole CPU count (nproc) -- the job is a share of the host, not all of it."""
    return {"job_cores": job_cores(), "sched_affinity": len(os.sched_getaffinity(0)),
            "OMP_NUM_THREADS": os.environ.get("OMP_NUM_THREADS"), "nproc": os.cpu_count()}


def cpu_baseline(args):
    """The reference's per-block sequence (ref.go:98-161: keyed BLAKE3 DEK,
    ChaCha20 XOR, BLAKE3 CID of the ctext, ctext into a buffer) timed on host
    cores over a bounded sample of the same workload (1 MiB blocks of the
    same stream).  value = the Go path's primitive mix on one core (the
    reference's Writer is single-goroutine, blob.go:71-83): SIMD BLAKE3
    (upstream C, AVX-512 -- as lukechampine.com/blake3's assembly, go.mod:12)
    with a portable scalar ChaCha20 (as x/crypto's generic Go ChaCha20, the
    one amd64 runs, go.mod:10) -- oracle_post_batch_gomix.  Beside it: the
    all-scalar oracle port, the all-SIMD libraries (OpenSSL ChaCha20), and
    the Go mix on the job's cores (job_cores) over independent block ranges."""
    from oracle import oracle as O
    L = O.lib()
    cores = job_cores()
    n = args.cpu_sample_mib * MIB
    n_all = 4 * n
    buf = ctypes.create_string_buffer(n_all)
    ct = ctypes.create_string_buffer(n_all)
    L.oracle_fill_splitmix(buf, 0, n_all, args.seed)
    refs = ctypes.create_string_buffer(64 * -(-n_all // args.block_size))
    salt = bytes(32)

    def timed(fn, nbytes, threads):
        t = time.perf_counter()
        rc = fn(refs, ct, salt, buf, nbytes, args.block_size, None, threads)
        dt = time.perf_counter() - t
        return (None if rc not in (None, 0) else nbytes / GIB / dt), dt

    go1, dgo1 = timed(L.oracle_post_batch_gomix, n, 1)
    port_n = max(MIB, n // 3)
    port1, dport1 = timed(L.oracle_post_batch, port_n, 1)
    goall, dgoall = timed(L.oracle_post_batch_gomix, n_all, cores)
    simd1, dsimd1 = timed(L.oracle_post_batch_simd, n, 1)
    simdall, dsimdall = timed(L.oracle_post_batch_simd, n_all, cores)
    del buf, ct
    model = ""
    try:
        with open("/proc/cpuinfo") as f:
            model = next((ln.split(":", 1)[1].strip() for ln in f
                          if ln.startswith("model name")), "")
    except OSError:
        pass
    r4 = lambda v: None if v is None else round(v, 4)
    if go1 is None:   # no SIMD BLAKE3 in this image: the all-scalar port
        go1, dgo1, kind_note = port1, dport1, "all-scalar port (no SIMD BLAKE3 found)"
    else:
        kind_note = "SIMD BLAKE3 + scalar ChaCha20 (the Go path's primitive mix)"
    return {"value": r4(go1), "unit": "GiB/s", "cores": 1, "kind": "port",
            "what": kind_note + ", one thread, same blocks and refs as the GPU",
            "sample": f"{args.cpu_sample_mib} MiB = {n // args.block_size} x "
                      f"{args.block_size // 1024} KiB blocks, oracle_post_batch_gomix, "
                      f"1 thread, {dgo1:.1f} s",
            "job_cores": {"value": r4(goall), "cores": cores,
                          "sample": f"{4 * args.cpu_sample_mib} MiB, {cores} threads over "
                                    f"independent block ranges, {dgoall:.1f} s"},
            "scalar_port": {"value": r4(port1), "cores": 1,
                            "sample": f"{port_n // MIB} MiB, oracle_post_batch (portable "
                                      f"scalar BLAKE3 and ChaCha20), {dport1:.1f} s"},
            "simd_libraries": {"value": r4(simd1), "cores": 1,
                               "job_cores": {"value": r4(simdall), "cores": cores},
                               "sample": f"upstream BLAKE3 C (AVX-512) + OpenSSL ChaCha20 "
                                         f"(AVX-512), {dsimd1:.1f} s / {dsimdall:.1f} s",
                               "what": "an upper bound for any per-core CPU path"},
            "host_cores": core_info(), "cpu_model": model}


def small_blobs(torch, N, stream, sp, n=1 << 20, ln=4096, reps=10):
    """BASELINE config 4's hashing: 1M distinct 4 KiB blobs (glfs.PostBlob with
    the blob type salt, bs = 2 MiB), device-resident, one lane per blob
    (glfsx_post_blobs_device).  Reported beside the headline, not as it."""
    from glfs_amd import glfs
    blob_salt = glfs.Machine().make_salt("blob")   # machine.go:50-54, on the GPU
    with torch.cuda.stream(stream):
        data = torch.empty(n * ln, dtype=torch.uint8, device="cuda")
        ct = torch.empty(n * ln, dtype=torch.uint8, device="cuda")
        roots = torch.empty(64 * n, dtype=torch.uint8, device="cuda")
        offs = torch.arange(n, dtype=torch.int64, device="cuda") * ln
        lens = torch.full((n,), ln, dtype=torch.int64, device="cuda")
        N.check(N.lib.glfsx_fill_splitmix_device(data.data_ptr(), 0, n * ln, 11, sp))
        ts = []
        for _ in range(reps + 1):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            N.check(N.lib.glfsx_post_blobs_device(2 << 20, blob_salt, None, data.data_ptr(),
                                                  offs.data_ptr(), lens.data_ptr(), n, ln,
                                                  ct.data_ptr(), roots.data_ptr(), sp))
            e1.record(stream)
            e1.synchronize()
            ts.append(e0.elapsed_time(e1))
    ms = sum(ts[1:]) / reps
    return {"value": round(n * ln / GIB / (ms * 1e-3), 2), "unit": "GiB/s",
            "blobs_per_s": round(n / (ms * 1e-3)), "ms": round(ms, 3),
            "reps": reps, "stat": "mean of the reps (HIP events on the launch stream)",
            "what": "1,048,576 distinct 4 KiB blobs, glfs.PostBlob roots (DEK + ChaCha20 "
                    "ctext to HBM + CID), one lane per blob"}


def small_blobs_from_host(torch, N, stream, sp, n=1 << 20, ln=4096, reps=3):
    """Config 4's hashing as a Go caller sees it (glfs.PostBlobs over
    glfsx_post_blobs): 1,048,576 distinct 4 KiB blobs
    (blob i = the splitmix stream of seed i) in pageable HOST memory, one
    glfsx_post_blobs call -- packed into pinned 64 MiB groups, uploaded,
    hashed one lane per blob, roots and ctext downloaded, every blob's Post
    delivered in order to a native sink -- PCIe inside the time.  The roots
    must equal the device-resident batch's."""
    import numpy as np
    from glfs_amd import glfs
    bs = 2 << 20
    salt = glfs.Machine().make_salt("blob")
    with torch.cuda.stream(stream):
        d = torch.empty(n * ln, dtype=torch.uint8, device="cuda")
        roots_d = torch.empty(64 * n, dtype=torch.uint8, device="cuda")
        offs_d = torch.arange(n, dtype=torch.int64, device="cuda") * ln
        lens_d = torch.full((n,), ln, dtype=torch.int64, device="cuda")
        N.check(N.lib.glfsx_fill_splitmix_blobs_device(d.data_ptr(), n, ln, 0, sp))
        N.check(N.lib.glfsx_post_blobs_device(bs, salt, None, d.data_ptr(), offs_d.data_ptr(),
                                              lens_d.data_ptr(), n, ln, None, roots_d.data_ptr(),
                                              sp))
    stream.synchronize()
    host = d.cpu().numpy()
    want = roots_d.cpu().numpy().tobytes()
    _GPU_REFS["small_blobs_seed0"] = want   # the CPU baseline checks its roots against these
    del d, roots_d, offs_d, lens_d
    offs = np.arange(n, dtype=np.uint64) * ln
    lens = np.full(n, ln, dtype=np.uint64)
    roots = np.empty(64 * n, dtype=np.uint8)
    counts = (ctypes.c_uint64 * 2)()
    sink = ctypes.cast(N.lib.glfsx_sink_count, N.POST_FN)
    res = {}
    for label, post in (("with_posts", sink), ("roots_only", N.POST_FN(0))):
        ts = []
        for _ in range(reps + 1):
            counts[0] = counts[1] = 0
            roots[:] = 0
            t = time.perf_counter()
            N.check(N.lib.glfsx_post_blobs(bs, bs, salt, None, host.ctypes.data, offs.ctypes.data,
                                           lens.ctypes.data, n, post, ctypes.byref(counts),
                                           roots.ctypes.data))
            ts.append(time.perf_counter() - t)
            assert roots.tobytes() == want, "host batch roots differ from the device batch"
            if label == "with_posts":
                assert counts[0] == n and counts[1] == n * ln, "sink missed Posts"
        sec = sum(ts[1:]) / reps
        res[label] = {"value": round(n * ln / GIB / sec, 2), "ms": round(sec * 1e3, 2),
                      "blobs_per_s": round(n / sec)}
    out = dict(res["with_posts"])
    out.update({"unit": "GiB/s", "reps": reps, "stat": "mean wall time after one warm-up call",
                "roots_only": res["roots_only"],
                "what": "1,048,576 x 4 KiB glfs blobs from pageable host memory through one "
                        "glfsx_post_blobs call (glfs.PostBlobs): pinned 64 MiB groups, H2D, "
                        "one lane per blob, roots + ctext D2H, every Post delivered in order "
                        "(native counting sink); roots_only: no sink, so no ctext download. "
                        "Roots equal the device batch's"})
    return out


_GPU_REFS = {}


def cpu_baseline_configs(args, config2_root_cid):
    """BASELINE.md section 2's other CPU baselines, the Go
    path's primitive mix (oracle_post_batch_gomix: SIMD BLAKE3 + scalar
    ChaCha20) on 1 core and on all cores of this job, each checked against
    the GPU's results:
      config2: BASELINE configs[1] -- a 1 GiB blob at 2 MiB blocks with the
        glfs blob salt (splitmix seed 1): 512 data posts with rawSalt, the
        index node with indexSalt (bigblob/ref.go:98-161, blob.go:165-206);
        the root must equal config2's GPU root.
      small_blobs: BASELINE config 4's hashing -- 1,048,576 x 4 KiB blobs
        (blob i = splitmix seed i), root = post(rawSalt, blob)
        (blob.go:190-193); 1 core over the first 262,144 blobs, all cores over
        all of them; the roots must equal the GPU's."""
    import hashlib
    from oracle import oracle as O
    L = O.lib()
    cores = job_cores()
    tsalt = O.derive_key(bytes(32), b"blob")            # machine.go:50-54
    raw, idx = O.derive_key(tsalt, b"raw"), O.derive_key(tsalt, b"index")
    out = {}
    # config 2
    size, bs = GIB, 2 * MIB
    buf = ctypes.create_string_buffer(size)
    ct = ctypes.create_string_buffer(size)
    L.oracle_fill_splitmix(buf, 0, size, 1)
    nb = size // bs
    refs = ctypes.create_string_buffer(64 * nb)
    c2 = {}
    for label, th in (("one_core", 1), ("job_cores", cores)):
        t = time.perf_counter()
        rc = L.oracle_post_batch_gomix(refs, ct, raw, buf, size, bs, None, th)
        root_ref, _ = O.post(idx, refs.raw.ljust(bs, b"\0"))   # the one index node
        dt = time.perf_counter() - t
        if rc not in (None, 0):
            c2 = {"error": "no SIMD BLAKE3 in this image"}
            break
        c2[label] = {"value": round(size / GIB / dt, 4), "cores": th, "s": round(dt, 2)}
        c2["root_equals_gpu"] = root_ref[:32].hex() == config2_root_cid
    c2.update({"unit": "GiB/s", "kind": "port",
               "sample": "the whole config: 1 GiB at 2 MiB blocks, 512 data posts + 1 index post"})
    out["config2"] = c2
    del buf, ct
    # config 4's hashing
    n, ln = 1 << 20, 4096
    buf = ctypes.create_string_buffer(n * ln)
    ct = ctypes.create_string_buffer(n * ln)
    L.oracle_fill_splitmix_blobs(buf, n, ln, 0)
    refs = ctypes.create_string_buffer(64 * n)
    want = _GPU_REFS.get("small_blobs_seed0")
    sb = {}
    for label, th, m in (("one_core", 1, n // 4), ("job_cores", cores, n)):
        t = time.perf_counter()
        rc = L.oracle_post_batch_gomix(refs, ct, raw, buf, m * ln, ln, None, th)
        dt = time.perf_counter() - t
        if rc not in (None, 0):
            sb = {"error": "no SIMD BLAKE3 in this image"}
            break
        got = refs.raw[:64 * m]
        sb[label] = {"value": round(m * ln / GIB / dt, 4), "blobs_per_s": round(m / dt),
                     "cores": th, "blobs": m, "s": round(dt, 2),
                     "roots_equal_gpu": (None if want is None else
                                         hashlib.sha256(got).digest() ==
                                         hashlib.sha256(want[:64 * m]).digest())}
    sb.update({"unit": "GiB/s", "kind": "port",
               "sample": "one_core: the first 262,144 of the 1,048,576 blobs; job_cores: all"})
    out["small_blobs"] = sb
    return out


def config2_leg(torch, N, stream, sp, steps=50, warmup=5):
    """BASELINE configs[1]: a 1 GiB blob at the glfs default block size
    (2 MiB, glfs.go:12) with the glfs blob type salt (machine.go:50-54, as
    glfs.PostBlob passes it to bigblob.NewWriter), data = the splitmix stream
    of seed 1 in HBM, ctext to HBM: 512 data posts + 1 index
    post per step.  Timed like the headline: HIP events around `steps`
    back-to-back Creates on the launch stream, mean per step."""
    from glfs_amd import glfs
    size, bs = GIB, 2 * MIB
    salt = glfs.Machine().make_salt("blob")
    with torch.cuda.stream(stream):
        data = torch.empty(size, dtype=torch.uint8, device="cuda")
        ct = torch.empty(size, dtype=torch.uint8, device="cuda")
        N.check(N.lib.glfsx_fill_splitmix_device(data.data_ptr(), 0, size, 1, sp))
    stream.synchronize()
    root, posts = N.glfsx_root(), ctypes.c_uint64()

    def step():
        N.check(N.lib.glfsx_create_device(bs, salt, None, data.data_ptr(), size,
                                          ct.data_ptr(), ctypes.byref(root),
                                          ctypes.byref(posts), sp))

    for _ in range(warmup):
        step()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t = time.perf_counter()
    e0.record(stream)
    for _ in range(steps):
        step()
    e1.record(stream)
    e1.synchronize()
    wall = (time.perf_counter() - t) / steps
    ms = e0.elapsed_time(e1) / steps
    del data, ct
    return {"value": round(size / GIB / (ms * 1e-3), 2), "unit": "GiB/s",
            "ms_per_step": round(ms, 4), "wall_ms_per_step": round(wall * 1e3, 4),
            "steps": steps, "warmup": warmup, "posts_per_step": posts.value,
            "root_cid": bytes(root.ref)[:32].hex(),
            "what": "BASELINE configs[1]: 1 GiB blob @ 2 MiB blocks (glfs default), glfs blob "
                    "salt, splitmix seed 1 in HBM, ctext to HBM; mean over steps (HIP events)"}


def config4_end_to_end(torch, N, stream, sp, n=1 << 20, ln=4096, reps=10, routes=None):
    """BASELINE config 4 end to end: 1,048,576 distinct 4 KiB blobs (blob i =
    splitmix stream of seed i) posted as glfs blobs (DEK + ChaCha20 ctext to
    HBM + CID per blob, machine.go:64), then the tree of them ("%07d" names,
    tree.go:250-260 PostTreeMap): its JSON lines encoded and the tree blob
    posted through the bigblob write path (2 MiB blocks + index node).
    Two routes, both timed from blobs resident in HBM to the tree root:
      device: roots stay in HBM, lines encoded on the GPU
              (glfsx_tree_encode_device), tree blob = glfsx_create_device;
      host:   roots copied to the host, lines encoded on host cores
              (glfsx_tree_encode, C++), tree blob through the Writer from
              host memory (glfsx_create, H2D + D2H of its ctext, counting
              sink).
    The per-entry ExistsUnit store lookup (tree.go:304) is the store's and
    is not in either route (the blobs were just posted).  value = blob bytes
    / time."""
    import numpy as np
    from glfs_amd import glfs
    bs = 2 << 20
    m = glfs.Machine()
    blob_salt, tree_salt = m.make_salt("blob"), m.make_salt("tree")
    cuda = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
    names_h = np.frombuffer("".join("%07d" % i for i in range(n)).encode(), dtype=np.uint8)
    name_offs_h = np.arange(n + 1, dtype=np.uint64) * 7
    types_h = np.frombuffer(b"blob" * n, dtype=np.uint8)
    type_offs_h = np.arange(n + 1, dtype=np.uint64) * 4
    modes_h = np.full(n, 0o644, dtype=np.uint32)
    sizes_h = np.full(n, ln, dtype=np.uint64)
    bss_h = np.full(n, bs, dtype=np.uint64)
    with torch.cuda.stream(stream):
        data = torch.empty(n * ln, dtype=torch.uint8, device="cuda")
        ct = torch.empty(n * ln, dtype=torch.uint8, device="cuda")
        roots = torch.empty(64 * n, dtype=torch.uint8, device="cuda")
        offs = torch.arange(n, dtype=torch.int64, device="cuda") * ln
        lens = torch.full((n,), ln, dtype=torch.int64, device="cuda")
        names = cuda(names_h)
        name_offs = cuda(name_offs_h.view(np.int64))
        types = cuda(types_h)
        type_offs = cuda(type_offs_h.view(np.int64))
        modes = cuda(modes_h.view(np.int32))
        bss = cuda(bss_h.view(np.int64))
        lines = torch.empty(260 * n, dtype=torch.uint8, device="cuda")
        tree_ct = torch.empty(260 * n, dtype=torch.uint8, device="cuda")
        N.check(N.lib.glfsx_fill_splitmix_blobs_device(data.data_ptr(), n, ln, 0, sp))
    stream.synchronize()
    roots_h = torch.empty(64 * n, dtype=torch.uint8).pin_memory()
    lines_h = np.empty(260 * n, dtype=np.uint8)
    total = ctypes.c_uint64()
    root = N.glfsx_root()
    counts = (ctypes.c_uint64 * 2)()
    sink = ctypes.cast(N.lib.glfsx_sink_count, N.POST_FN)

    def post_blobs():
        N.check(N.lib.glfsx_post_blobs_device(bs, blob_salt, None, data.data_ptr(),
                                              offs.data_ptr(), lens.data_ptr(), n, ln,
                                              ct.data_ptr(), roots.data_ptr(), sp))

    def host_route():
        post_blobs()
        with torch.cuda.stream(stream):
            roots_h.copy_(roots, non_blocking=True)
        stream.synchronize()
        N.check(N.lib.glfsx_tree_encode(n, names_h.ctypes.data, name_offs_h.ctypes.data,
                                        modes_h.ctypes.data, types_h.ctypes.data,
                                        type_offs_h.ctypes.data, roots_h.data_ptr(),
                                        sizes_h.ctypes.data, bss_h.ctypes.data,
                                        lines_h.ctypes.data, lines_h.size,
                                        ctypes.byref(total), None))
        counts[0] = counts[1] = 0
        N.check(N.lib.glfsx_create(bs, bs, tree_salt, None, lines_h.ctypes.data, total.value,
                                   sink, ctypes.byref(counts), ctypes.byref(root)))
        return bytes(root.ref)

    # the device route's pieces, HIP events on the launch stream in the same
    # reps as its wall time: post_blobs | tree lines | tree Create
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]

    def device_route_timed():
        ev[0].record(stream)
        post_blobs()
        ev[1].record(stream)
        N.check(N.lib.glfsx_tree_encode_device(n, names.data_ptr(), name_offs.data_ptr(),
                                               modes.data_ptr(), types.data_ptr(),
                                               type_offs.data_ptr(), roots.data_ptr(),
                                               lens.data_ptr(), bss.data_ptr(),
                                               lines.data_ptr(), lines.numel(), None,
                                               ctypes.byref(total), sp))
        ev[2].record(stream)
        N.check(N.lib.glfsx_create_device(bs, tree_salt, None, lines.data_ptr(), total.value,
                                          tree_ct.data_ptr(), ctypes.byref(root), None, sp))
        ev[3].record(stream)
        return bytes(root.ref)

    roots2 = torch.empty(64 * n, dtype=torch.uint8, device="cuda")

    def one_call_route():
        # glfsx_post_tree_device: blob hashing, lines and the tree blob
        # overlapped (the lines' layout beside the hashing, tree blocks
        # posted on a second stream as their bytes are written)
        N.check(N.lib.glfsx_post_tree_device(n, bs, blob_salt, tree_salt, None, data.data_ptr(),
                                             offs.data_ptr(), lens.data_ptr(), ln, ct.data_ptr(),
                                             roots2.data_ptr(), names.data_ptr(),
                                             name_offs.data_ptr(), modes.data_ptr(),
                                             types.data_ptr(), type_offs.data_ptr(),
                                             bss.data_ptr(), bs, lines.data_ptr(), lines.numel(),
                                             tree_ct.data_ptr(), ctypes.byref(root),
                                             ctypes.byref(total), sp))
        return bytes(root.ref)

    res = {}
    for name, fn in (("device", device_route_timed), ("one_call", one_call_route),
                     ("host", host_route)):
        if routes is not None and name not in routes:
            continue
        fn()
        ts, parts = [], []
        for _ in range(reps):
            stream.synchronize()
            t = time.perf_counter()
            r = fn()
            stream.synchronize()
            ts.append(time.perf_counter() - t)
            if name == "device":
                parts.append([ev[k].elapsed_time(ev[k + 1]) for k in range(3)])
        sec = sum(ts) / reps
        res[name] = {"value": round(n * ln / GIB / sec, 2), "unit": "GiB/s",
                     "ms": round(sec * 1e3, 3), "blobs_per_s": round(n / sec),
                     "reps": reps, "stat": "mean wall time over the reps",
                     "min_ms": round(min(ts) * 1e3, 3),
                     "tree_bytes": total.value, "tree_root_cid": r[:32].hex()}
        if parts:
            mean = [sum(p[k] for p in parts) / reps for k in range(3)]
            res[name]["pieces_ms"] = {"post_blobs": round(mean[0], 3),
                                      "tree_lines": round(mean[1], 3),
                                      "tree_create": round(mean[2], 3)}
            res[name]["gpu_ms"] = round(sum(mean), 3)
            res[name]["host_gaps_ms"] = round(sec * 1e3 - sum(mean), 3)
            res[name]["pieces_what"] = ("means of HIP events on the launch stream in the same "
                                        "reps; wall = gpu_ms + host_gaps_ms (launch and sync "
                                        "overheads between the pieces)")
    if routes is not None:   # a subset for profiling (scripts/legs.py config4one)
        return res
    assert res["device"]["tree_root_cid"] == res["host"]["tree_root_cid"]
    assert res["one_call"]["tree_root_cid"] == res["host"]["tree_root_cid"]
    out = dict(res["one_call"])
    out["what"] = ("1,048,576 x 4 KiB glfs blobs (HBM) -> roots -> PostTreeMap JSON lines "
                   "(\"%07d\" names) -> tree blob root, one glfsx_post_tree_device call "
                   "(blob hashing, lines on the GPU and the tree blob overlapped); value = "
                   "blob bytes / time")
    out["three_calls"] = res["device"]
    out["three_calls"]["what"] = ("same as glfsx_post_blobs_device, glfsx_tree_encode_device, "
                                  "glfsx_create_device in sequence, with the pieces' times")
    out["host_encode_route"] = res["host"]
    out["host_encode_route"]["what"] = ("same, roots D2H, lines on host cores "
                                        "(glfsx_tree_encode), tree via the Writer from host")
    return out


def host_round_trip(N, args, bs, barrier=lambda: None, slowest=lambda s: s):
    """Host memory -> GPU -> host: glfsx_create over a pageable host buffer with
    a store sink that receives every ctext + ref on the host (blob.go Writer
    semantics).  PCIe-inclusive; never the headline value."""
    import numpy as np
    n = int(args.host_rt_gib * GIB) // bs * bs
    if n == 0:
        return None
    import torch
    # the same splitmix stream, generated on the GPU and copied down
    host = host_stream(torch, N, n, args.seed)
    root = N.glfsx_root()

    def run(sink, ctx, check):
        best = None
        for _ in range(3):
            c = ctx()
            barrier()
            t = time.perf_counter()
            N.check(N.lib.glfsx_create(bs, bs, None, None, host.ctypes.data, n, sink, c,
                                       ctypes.byref(root)))
            dt = slowest(time.perf_counter() - t)
            check(c)
            best = dt if best is None else min(best, dt)
        return round(n / GIB / best, 2)

    counts = (ctypes.c_uint64 * 2)()

    def count_ctx():
        counts[0] = counts[1] = 0
        return ctypes.byref(counts)

    def count_check(_):
        assert counts[1] >= n and counts[0] > n // bs, "sink did not see every block"

    stores = []

    def store_ctx(mode, keep):
        def make():
            while stores:
                N.lib.glfsx_store_free(stores.pop())
            s = N.lib.glfsx_store_new(bs, mode, 0, keep, None)
            assert s, "native store unavailable"
            stores.append(s)
            return ctypes.c_void_p(s)
        return make

    def store_check(c):
        posts = ctypes.c_uint64()
        N.lib.glfsx_store_stats(c, ctypes.byref(posts), None, None)
        assert posts.value > n // bs

    count_sink = ctypes.cast(N.lib.glfsx_sink_count, N.POST_FN)   # native, no Python per block
    store_post = ctypes.cast(N.lib.glfsx_store_post, N.POST_FN)
    res = {"count_sink": run(count_sink, count_ctx, count_check)}
    want_root = bytes(root.ref)
    res["trusting_store"] = run(store_post, store_ctx(N.GLFSX_STORE_TRUST, 0), store_check)
    res["hashing_store"] = run(store_post, store_ctx(N.GLFSX_STORE_HASH, 0), store_check)
    res["trusting_store_keeping_bytes"] = run(store_post, store_ctx(N.GLFSX_STORE_TRUST, 1),
                                              store_check)

    def io_copy(strict, piece):
        """Create as bigblob does it: io.Copy(w, r) into the Writer in
        `piece`-byte writes (glfs.go:53, blob.go:213), pre-hashed store."""
        best = None
        for _ in range(3):
            c = store_ctx(N.GLFSX_STORE_TRUST, 0)()
            err = ctypes.c_int()
            barrier()
            t = time.perf_counter()
            w = N.lib.glfsx_writer_new(bs, bs, None, None, store_post, c, ctypes.byref(err))
            assert w, N.last_error()
            N.check(N.lib.glfsx_writer_set_strict(w, int(strict)))
            rc = N.lib.glfsx_writer_copy(w, host.ctypes.data, n, piece)
            if rc == 0:
                rc = N.lib.glfsx_writer_finish(w, ctypes.byref(root))
            msg = (N.lib.glfsx_writer_error(w) or b"").decode()
            N.lib.glfsx_writer_free(w)
            dt = slowest(time.perf_counter() - t)
            N.check(rc, msg)
            store_check(c)
            best = dt if best is None else min(best, dt)
        return round(n / GIB / best, 2)

    def read_from(piece, strict=False):
        """io.Copy through the Writer's ReadFrom (glfsx_writer_reserve /
        _commit): a reader that copies up to `piece` bytes per Read straight
        into the pinned staging (one thread, like read(2) from a file).
        strict: the Go binding's default writer (GLFSX_STRICT=1), whose
        ReadFrom turns strict off for its batches, then back on and flushes
        before returning (integration/go/gpu.go ReadFrom)."""
        best = None
        buf, cap = ctypes.c_void_p(), ctypes.c_uint64()
        for _ in range(3):
            c = store_ctx(N.GLFSX_STORE_TRUST, 0)()
            err = ctypes.c_int()
            barrier()
            t = time.perf_counter()
            w = N.lib.glfsx_writer_new(bs, bs, None, None, store_post, c, ctypes.byref(err))
            assert w, N.last_error()
            off, rc = 0, 0
            if strict:
                N.check(N.lib.glfsx_writer_set_strict(w, 1))
                N.check(N.lib.glfsx_writer_set_strict(w, 0))   # ReadFrom's entry
            while rc == 0 and off < n:
                rc = N.lib.glfsx_writer_reserve(w, ctypes.byref(buf), ctypes.byref(cap))
                if rc == 0:
                    k = min(cap.value, piece, n - off)
                    ctypes.memmove(buf.value, host.ctypes.data + off, k)
                    rc = N.lib.glfsx_writer_commit(w, k)
                    off += k
            if rc == 0 and strict:   # ReadFrom's return
                N.check(N.lib.glfsx_writer_set_strict(w, 1))
                rc = N.lib.glfsx_writer_flush(w)
            if rc == 0:
                rc = N.lib.glfsx_writer_finish(w, ctypes.byref(root))
            msg = (N.lib.glfsx_writer_error(w) or b"").decode()
            N.lib.glfsx_writer_free(w)
            dt = slowest(time.perf_counter() - t)
            N.check(rc, msg)
            store_check(c)
            best = dt if best is None else min(best, dt)
        return round(n / GIB / best, 2)

    res["io_copy_32k_pipelined"] = io_copy(False, 32 << 10)
    res["io_copy_32k_strict"] = io_copy(True, 32 << 10)
    res["read_from_1m"] = read_from(MIB)
    res["read_from_64m"] = read_from(64 * MIB)
    res["read_from_1m_strict"] = read_from(MIB, strict=True)
    while stores:
        N.lib.glfsx_store_free(stores.pop())
    home = int(torch.cuda.current_device())
    ff = file_feed(N, host, bs, {"lanes_1": [home], "lanes_3": [home] * 3}, want_root)
    res["file_read_fd"] = ff["lanes_1"]
    res["file_read_fd_3_lanes"] = ff["lanes_3"]
    return {"value": res["trusting_store"], "unit": "GiB/s", "bytes": n,
            "what": "glfsx_create (bigblob Writer) from pageable host memory: staging copy, "
                    "H2D, kernels, D2H of every ctext + ref, each Post delivered in order to "
                    "a native pre-hashed store (glfsx_store, GLFSX_STORE_TRUST: takes the GPU "
                    "CID, keeps CIDs); upload / hash / download on three streams",
            "sinks": res,
            "sinks_what": {
                "count_sink": "Posts only counted (the pipeline's PCIe ceiling)",
                "trusting_store": "pre-hashed Post: the store keeps the GPU CID, no host hash",
                "hashing_store": "today's drop-in: the store re-hashes every ctext with "
                                 "BLAKE3 on the Writer's thread (ref.go:103 MemStore.Post; "
                                 "upstream BLAKE3 C, AVX-512, 1 core)",
                "trusting_store_keeping_bytes": "pre-hashed Post into a store that copies "
                                                "every ctext (MemStore's memory cost)",
                "io_copy_32k_pipelined": "bigblob.Create fed by io.Copy's 32 KiB Writes "
                                         "(glfs.go:53; a reader that is not a WriterTo, "
                                         "into a Writer without ReadFrom), pipelined 64 MiB "
                                         "batches, pre-hashed store",
                "io_copy_32k_strict": "the same with blob.go:120-133 error timing "
                                      "(GLFSX_STRICT=1): every Write that completes a block "
                                      "returns after its Post (one-shot post per block)",
                "read_from_1m": "io.Copy through the Writer's ReadFrom (glfsx_writer_reserve"
                                "/_commit): the reader copies 1 MiB per Read straight into "
                                "the pinned staging (one thread, no second copy)",
                "read_from_64m": "the same with 64 MiB Reads",
                "read_from_1m_strict": "read_from_1m on a strict writer, the Go binding's "
                                       "default (GLFSX_STRICT=1): ReadFrom pipelines its "
                                       "batches and flushes their Posts before returning",
                "file_read_fd": ff["what"] + " (one lane)",
                "file_read_fd_3_lanes": "the same, the Writer's batches over 3 lanes of the "
                                        "one GPU ([0, 0, 0]: shared streams, more slots in "
                                        "flight)"}}


def one_process_multi_gpu(torch, N, args, world, bs, home):
    """The multi-GPU write path from ONE process over `world` GPUs (what a
    Go process on this node calls through the C-ABI): glfsx_create_devices
    over bf-aligned 16 GiB parts, one per GPU, device-resident (each part's
    data blocks and level-1 nodes on its GPU, levels >= 2 on the first),
    and one Writer fed from one pageable host stream with its batches
    round-robin over every GPU (glfsx_writer_set_devices) into the
    pre-hashed store."""
    import numpy as np
    ndev = torch.cuda.device_count()
    # one GPU per rank; fewer GPUs than ranks only when rehearsing on one box
    devs = [k % ndev for k in range(world)]
    bf = bs // 64
    part = bs * bf                       # 16 GiB at 1 MiB: one level-1 node
    bufs = []
    for k, d in enumerate(devs):
        N.set_device(d)
        t = torch.empty(part, dtype=torch.uint8, device=f"cuda:{d}")
        N.check(N.lib.glfsx_fill_splitmix_device(t.data_ptr(), k * part, part, args.seed, None))
        bufs.append(t)
    for d in devs:
        torch.cuda.synchronize(d)
    N.set_device(home)
    nd = len(devs)
    cdevs = (ctypes.c_int * nd)(*devs)
    ptrs = (ctypes.c_void_p * nd)(*[t.data_ptr() for t in bufs])
    sizes = (ctypes.c_uint64 * nd)(*([part] * nd))
    root, posts = N.glfsx_root(), ctypes.c_uint64()

    def create():
        N.check(N.lib.glfsx_create_devices(bs, None, None, nd, cdevs, ptrs, sizes, None, None,
                                           ctypes.byref(root), ctypes.byref(posts)))

    create()
    reps = 5
    t = time.perf_counter()
    for _ in range(reps):
        create()
    sec = (time.perf_counter() - t) / reps
    dev_res = {"value": round(nd * part / GIB / sec, 2), "unit": "GiB/s",
               "ms_per_create": round(sec * 1e3, 3), "gpus": nd, "part_bytes": part,
               "posts": posts.value, "root_cid": bytes(root.ref)[:32].hex(),
               "what": f"glfsx_create_devices, {nd} x {part // GIB} GiB parts in HBM "
                       "(ctext not written), mean of 5 Creates, host wall clock"}
    del bufs
    # one host stream over all GPUs
    per = int(min(args.host_rt_gib, 4.0) * GIB) // bs * bs
    host_res = None
    if per > 0:
        n = per * nd
        host = np.empty(n, dtype=np.uint8)
        tmp = torch.empty(64 * MIB, dtype=torch.uint8, device=f"cuda:{home}")
        for off in range(0, n, 64 * MIB):
            m = min(64 * MIB, n - off)
            N.check(N.lib.glfsx_fill_splitmix_device(tmp.data_ptr(), off, m, args.seed, None))
            torch.cuda.synchronize()
            host[off:off + m] = tmp[:m].cpu().numpy()
        del tmp
        store_post = ctypes.cast(N.lib.glfsx_store_post, N.POST_FN)
        best = {}
        for label, lanes in (("one_gpu", devs[:1]), ("all_gpus", devs)):
            for _ in range(3):
                st = N.lib.glfsx_store_new(bs, N.GLFSX_STORE_TRUST, 0, 0, None)
                err = ctypes.c_int()
                t = time.perf_counter()
                w = N.lib.glfsx_writer_new(bs, bs, None, None, store_post, st, ctypes.byref(err))
                assert w, N.last_error()
                rc = N.lib.glfsx_writer_set_devices(w, (ctypes.c_int * len(lanes))(*lanes),
                                                    len(lanes))
                if rc == 0:
                    rc = N.lib.glfsx_writer_copy(w, host.ctypes.data, n, 64 * MIB)
                if rc == 0:
                    rc = N.lib.glfsx_writer_finish(w, ctypes.byref(root))
                msg = (N.lib.glfsx_writer_error(w) or b"").decode()
                N.lib.glfsx_writer_free(w)
                dt = time.perf_counter() - t
                N.lib.glfsx_store_free(st)
                N.check(rc, msg)
                best[label] = min(best.get(label, dt), dt)
        host_res = {"value": round(n / GIB / best["all_gpus"], 2), "unit": "GiB/s",
                    "one_gpu_value": round(n / GIB / best["one_gpu"], 2), "bytes": n,
                    "root_cid": bytes(root.ref)[:32].hex(),
                    "what": f"one Writer, one pageable host stream of {n // GIB} GiB in 64 MiB "
                            f"writes, batches round-robin over {nd} GPUs (glfsx_writer_set_"
                            "devices), pre-hashed store; one_gpu_value: the same on the first "
                            "GPU only; best of 3"}
    return {"device_resident": dev_res, "host_stream": host_res}


def postblob_latency(N, calls=300):
    """glfs.PostBlob as the drop-in runs it per blob (machine.go:64: one
    Writer, glfsx_create with the blob type salt at bs 2 MiB, a counting
    sink): per-call p50 / p90 from one thread (through ctypes; the C harness
    scripts/latency.c also measures concurrent callers)."""
    import numpy as np
    from glfs_amd import glfs
    salt = glfs.Machine().make_salt("blob")
    sink = ctypes.cast(N.lib.glfsx_sink_count, N.POST_FN)
    counts, root = (ctypes.c_uint64 * 2)(), N.glfsx_root()
    res = {}
    for size in (0, 4096, 65536, MIB, 2 * MIB):
        data = np.frombuffer(np.random.default_rng(size).bytes(max(size, 1)), dtype=np.uint8)
        ts = []
        for i in range(calls + 20):
            t = time.perf_counter()
            N.check(N.lib.glfsx_create(2 * MIB, 2 * MIB, salt, None, data.ctypes.data, size,
                                       sink, ctypes.byref(counts), ctypes.byref(root)))
            if i >= 20:
                ts.append(time.perf_counter() - t)
        ts.sort()
        res[str(size)] = {"p50_us": round(ts[len(ts) // 2] * 1e6, 1),
                          "p90_us": round(ts[int(len(ts) * 0.9)] * 1e6, 1)}
    return {"unit": "us per call", "calls": calls, "by_blob_bytes": res,
            "what": "one glfs.PostBlob (glfsx_create, bs 2 MiB, blob type salt, counting "
                    "sink) from one Python thread: staging copy, one-shot GPU post "
                    "(k_one / k_med_*), wait"}


def postblob_concurrency(N, ln=4096, plan=((1, 3000), (16, 1500), (64, 600), (256, 200))):
    """glfs.PostBlob as concurrent Go callers run it (VERDICT r4 next #5;
    glfsposix.go:49 ParMapErr posts one file per call, machine.go:64): T
    plain C threads (tools/libpostbench.so; no interpreter between calls),
    each posting its own distinct 4 KiB blobs one glfsx_create at a time
    (bs 2 MiB, blob type salt, counting sink).  calls/s = all calls / wall
    time; the CPU port's per-blob rate on 1 core and on all cores of this
    job is cpu_baseline.small_blobs (the same 4 KiB posts as a batch, no
    call overhead)."""
    from glfs_amd import glfs
    lib = ctypes.CDLL(os.path.join(ROOT, "tools", "libpostbench.so"))
    lib.postbench_run.restype = ctypes.c_int
    lib.postbench_run.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_int, ctypes.c_uint64,
                                                           ctypes.c_int, ctypes.c_char_p,
                                                           ctypes.c_int, ctypes.c_void_p]
    fns = [ctypes.cast(getattr(N.lib, f), ctypes.c_void_p).value
           for f in ("glfsx_create", "glfsx_set_device", "glfsx_sink_count")]
    salt = glfs.Machine().make_salt("blob")
    import torch
    dev = int(torch.cuda.current_device())
    res = {}
    stats = (ctypes.c_uint64 * 3)()
    for threads, calls in plan:
        out = (ctypes.c_double * 5)()
        N.check(N.lib.glfsx_one_stats(1, None))
        rc = lib.postbench_run(*fns, threads, ln, calls, salt, dev, out)
        N.check(rc, "postbench")
        N.check(N.lib.glfsx_one_stats(1, stats))
        res[str(threads)] = {"calls_per_s": round(out[0] / out[1]), "calls": int(out[0]),
                             "p50_us": round(out[2], 1), "p90_us": round(out[3], 1),
                             "p99_us": round(out[4], 1), "launches": int(stats[0]),
                             "mean_batch": round(stats[1] / max(stats[0], 1), 2),
                             "lanes_full": int(stats[2])}
    return {"by_threads": res, "blob_bytes": ln,
            "what": "concurrent glfs.PostBlob of distinct 4 KiB blobs: T C threads each calling "
                    "glfsx_create back to back (bs 2 MiB, blob type salt, counting sink); "
                    "calls_per_s = calls / wall time, latency percentiles per call; launches / "
                    "mean_batch / lanes_full from glfsx_one_stats (group commit: requests per "
                    "launch, leader found all 8 launch lanes busy), warm-up calls included"}


def concat_leg(N, bs=MIB, size=GIB):
    """blob.go:333-345 Concat of one 1 GiB blob in a native store: the read
    side (index level + every data block, one batched GPU decrypt per level,
    from host memory) feeding a new Writer (GPU hash, Posts into the store).
    Host round trip both ways; timed end to end."""
    import numpy as np
    from glfs_amd import bigblob
    import torch
    src = np.empty(size, dtype=np.uint8)
    dev = torch.empty(64 * MIB, dtype=torch.uint8, device="cuda")
    for off in range(0, size, 64 * MIB):
        N.check(N.lib.glfsx_fill_splitmix_device(dev.data_ptr(), off, 64 * MIB, 21, None))
        torch.cuda.synchronize()
        src[off:off + 64 * MIB] = dev.cpu().numpy()
    del dev
    st = bigblob.NativeStore(bs, "trust")
    m = bigblob.Machine(bs)
    root = m.create(st, None, memoryview(src))
    m.concat(st, bs, None, root)          # warm-up
    ts = []
    for _ in range(3):
        t = time.perf_counter()
        r2 = m.concat(st, bs, None, root)
        ts.append(time.perf_counter() - t)
    assert r2.ref == root.ref and r2.size == size
    sec = sum(ts) / len(ts)
    return {"value": round(size / GIB / sec, 2), "unit": "GiB/s", "ms": round(sec * 1e3, 1),
            "reps": 3, "stat": "mean wall time after one warm-up",
            "what": "bigblob Concat of a 1 GiB blob (1 MiB blocks) in a native store: index "
                    "level decrypted in one batch, data blocks handed to the new Writer as "
                    "ciphertext straight from the store's memory (64 MiB slabs gathered by "
                    "the copy threads into two pinned buffers in turn) and decrypted on the "
                    "GPU into its staging (glfsx_writer_write_ctext_blocks); Python API"}


if __name__ == "__main__":
    main()

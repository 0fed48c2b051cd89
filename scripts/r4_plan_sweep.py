"""Split-plan sweep (round 4): time glfsx_create_device for the config-4 tree
blob shape (241,172,480 B at 2 MiB blocks: 115 blocks + 1 index node, tree
salt) and config 2 (1 GiB at 2 MiB, blob salt) under several split targets
(glfsx_set_split_target: workgroups per launch below which a block is spread
over more workgroups with fewer chunks per lane).  HIP events on the launch
stream, mean of reps, interleaved."""
import ctypes
import json
import sys

import torch

sys.path.insert(0, ".")
from glfs_amd import _native as N, glfs  # noqa: E402

GIB, MIB = 1 << 30, 1 << 20
m = glfs.Machine()
shapes = {"tree_blob": (241172480, 2 * MIB, m.make_salt("tree")),
          "config2": (GIB, 2 * MIB, m.make_salt("blob"))}
args = sys.argv[1:]
if args and args[0] == "--shapes":   # --shapes NxBS,NxBS,... (blocks x block size)
    shapes = {}
    for sh in args[1].split(","):
        nb, bs = (int(x) for x in sh.split("x"))
        shapes[f"{nb}x{bs >> 10}K"] = (nb * bs, bs, m.make_salt("blob"))
    args = args[2:]
targets = [int(x) for x in (args or ["2048", "1024", "512", "400", "256", "128"])]
stream = torch.cuda.Stream()
sp = ctypes.c_void_p(stream.cuda_stream)
res = {k: {t: [] for t in targets} for k in shapes}
roots = {}
bufs = {}
with torch.cuda.stream(stream):
    for k, (size, bs, salt) in shapes.items():
        d = torch.empty(size, dtype=torch.uint8, device="cuda")
        c = torch.empty(size, dtype=torch.uint8, device="cuda")
        N.check(N.lib.glfsx_fill_splitmix_device(d.data_ptr(), 0, size, 1, sp))
        bufs[k] = (d, c)
stream.synchronize()
root = N.glfsx_root()
for rep in range(4):
    for t in targets:
        N.set_split_target(t)
        for k, (size, bs, salt) in shapes.items():
            d, c = bufs[k]
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            for _ in range(3):   # warm
                N.check(N.lib.glfsx_create_device(bs, salt, None, d.data_ptr(), size, c.data_ptr(),
                                                  ctypes.byref(root), None, sp))
            e0.record(stream)
            for _ in range(20):
                N.check(N.lib.glfsx_create_device(bs, salt, None, d.data_ptr(), size, c.data_ptr(),
                                                  ctypes.byref(root), None, sp))
            e1.record(stream)
            e1.synchronize()
            res[k][t].append(e0.elapsed_time(e1) / 20)
            r = bytes(root.ref).hex()
            assert roots.setdefault(k, r) == r, (k, t)
N.set_split_target(2048)
out = {}
for k, (size, bs, salt) in shapes.items():
    out[k] = {t: {"ms": round(sum(v[1:]) / len(v[1:]), 4),
                  "GiBps": round(size / GIB / (sum(v[1:]) / len(v[1:]) * 1e-3), 1)}
              for t, v in res[k].items()}
print(json.dumps(out, indent=1))

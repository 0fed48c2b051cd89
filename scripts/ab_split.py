"""A/B of the split target (glfsx_set_split_target) in one process,
interleaved: config 2 (1 GiB at 2 MiB blocks) and a 64 MiB blob at 1 MiB,
device-resident, ctext to HBM; prints GiB/s per (target, workload, rep).
usage: python scripts/ab_split.py 2048 1024 ..."""
import ctypes
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from glfs_amd import _native as N  # noqa: E402

GIB = 1 << 30
targets = [int(t) for t in sys.argv[1:]] or [2048, 1024]
N.set_device(0)
stream = torch.cuda.Stream()
sp = ctypes.c_void_p(stream.cuda_stream)
work = [("config2", 1 << 30, 2 << 20, 40), ("64MiB", 64 << 20, 1 << 20, 200)]
bufs = {}
with torch.cuda.stream(stream):
    for name, size, bs, _ in work:
        d = torch.empty(size, dtype=torch.uint8, device="cuda")
        c = torch.empty(size, dtype=torch.uint8, device="cuda")
        N.check(N.lib.glfsx_fill_splitmix_device(d.data_ptr(), 0, size, 1, sp))
        bufs[name] = (d, c)
stream.synchronize()
root = N.glfsx_root()
n_posts = ctypes.c_uint64()
roots = {}
for rep in range(3):
    for t in targets:
        N.set_split_target(t)
        for name, size, bs, steps in work:
            d, c = bufs[name]

            def step():
                N.check(N.lib.glfsx_create_device(bs, None, None, d.data_ptr(), size,
                                                  c.data_ptr(), ctypes.byref(root),
                                                  ctypes.byref(n_posts), sp))
            for _ in range(3):
                step()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(steps):
                step()
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            r = bytes(root.ref)
            assert roots.setdefault(name, r) == r, "root differs between targets"
            print(f"{rep} target {t:5d} {name:8s} {size / GIB * steps / dt:8.2f} GiB/s",
                  flush=True)

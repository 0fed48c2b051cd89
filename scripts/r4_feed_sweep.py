"""File-feed sensitivity (round 4): bigblob.Create from a 4 GiB tmpfs file
through glfsx_writer_read_fd into a pre-hashed store, best of 3, for the
GLFSX_READ_THREADS / GLFSX_SLOTS / GLFSX_BATCH_MIB settings in the
environment; also the pageable-memory Create (count sink) as the box's PCIe
ceiling.  Prints one JSON line.  usage: K=V ... python scripts/r4_feed_sweep.py"""
import ctypes
import json
import os
import sys
import tempfile
import time

import torch

sys.path.insert(0, ".")
import bench  # noqa: E402
from glfs_amd import _native as N  # noqa: E402

GIB, MIB = 1 << 30, 1 << 20
bs, n = MIB, 4 * GIB
bound = None
if os.environ.get("FEED_NUMA") == "1":   # run on the GPU's NUMA node
    bound = bench.numa_bind(torch, 0)
host = bench.host_stream(torch, N, n, 3)
root = N.glfsx_root()
counts = (ctypes.c_uint64 * 2)()
sink = ctypes.cast(N.lib.glfsx_sink_count, N.POST_FN)
best = None
for _ in range(3):
    t = time.perf_counter()
    N.check(N.lib.glfsx_create(bs, bs, None, None, host.ctypes.data, n, sink, ctypes.byref(counts),
                               ctypes.byref(root)))
    dt = time.perf_counter() - t
    best = dt if best is None else min(best, dt)
want = bytes(root.ref)
res = {"env": {k: v for k, v in os.environ.items() if k.startswith(("GLFSX_", "FEED_"))},
       "numa_node": bound,
       "pageable_count_sink": round(n / GIB / best, 2)}
res.update(bench.file_feed(N, host, bs, {"lanes_1": [0]}, want))
res.pop("what", None)
print(json.dumps(res), flush=True)

"""Host round-trip diagnostic: glfsx_create from a host buffer with the native
counting sink (same as bench.py's host_round_trip leg)."""
import ctypes
import sys
import time

import numpy as np

sys.path.insert(0, ".")
from glfs_amd import _native as N  # noqa: E402

gib = float(sys.argv[1]) if len(sys.argv) > 1 else 4
hold = float(sys.argv[2]) if len(sys.argv) > 2 else 0   # GiB held by torch's allocator
if hold:
    import torch
    held = [torch.empty(int(hold * (1 << 30)), dtype=torch.uint8, device="cuda")]
    if len(sys.argv) > 3 and sys.argv[3] == "free":
        del held
bs = 1 << 20
n = int(gib * (1 << 30)) // bs * bs
host = np.ones(n, dtype=np.uint8)
counts = (ctypes.c_uint64 * 2)()
sink = ctypes.cast(N.lib.glfsx_sink_count, N.POST_FN)
root = N.glfsx_root()
for _ in range(3):
    t = time.perf_counter()
    N.check(N.lib.glfsx_create(bs, bs, None, None, host.ctypes.data, n, sink,
                               ctypes.byref(counts), ctypes.byref(root)))
    dt = time.perf_counter() - t
    print(f"{n / dt / 2**30:.2f} GiB/s ({dt * 1e3:.1f} ms)", flush=True)

"""Writer lanes A/B on one GPU: the same 4 GiB pageable stream through one
Writer with its batches on lanes [0], [0, 0], [0, 0, 0] (glfsx_writer_set_
devices), counting sink and pre-hashed store, best of 3 each; plus 32 KiB
writes (io.Copy) on one lane, pipelined and strict.
usage: python scripts/lanes.py [GiB]"""
import ctypes
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
from glfs_amd import _native as N  # noqa: E402

MIB, GIB = 1 << 20, 1 << 30
gib = float(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1] != "-v" else 4.0
bs = MIB
n = int(gib * GIB)
host = np.empty(n, dtype=np.uint8)
tmp = torch.empty(64 * MIB, dtype=torch.uint8, device="cuda")
for off in range(0, n, 64 * MIB):
    m = min(64 * MIB, n - off)
    N.check(N.lib.glfsx_fill_splitmix_device(tmp.data_ptr(), off, m, 3, None))
    torch.cuda.synchronize()
    host[off:off + m] = tmp[:m].cpu().numpy()
count = ctypes.cast(N.lib.glfsx_sink_count, N.POST_FN)
store_post = ctypes.cast(N.lib.glfsx_store_post, N.POST_FN)
root = N.glfsx_root()


def run(lanes, sink_kind, piece, strict=False, reps=3):
    best, all_ = None, []
    for _ in range(reps):
        counts = (ctypes.c_uint64 * 2)()
        st = N.lib.glfsx_store_new(bs, N.GLFSX_STORE_TRUST, 0, 0, None)
        sink, ctx = (count, ctypes.byref(counts)) if sink_kind == "count" else \
            (store_post, ctypes.c_void_p(st))
        err = ctypes.c_int()
        t = time.perf_counter()
        w = N.lib.glfsx_writer_new(bs, bs, None, None, sink, ctx, ctypes.byref(err))
        if lanes is not None:
            N.check(N.lib.glfsx_writer_set_devices(w, (ctypes.c_int * len(lanes))(*lanes),
                                                   len(lanes)))
        N.lib.glfsx_writer_set_strict(w, int(strict))
        rc = N.lib.glfsx_writer_copy(w, host.ctypes.data, n, piece)
        rc = rc or N.lib.glfsx_writer_finish(w, ctypes.byref(root))
        N.lib.glfsx_writer_free(w)
        dt = time.perf_counter() - t
        N.lib.glfsx_store_free(st)
        N.check(rc)
        all_.append(round(n / GIB / dt, 1))
        best = dt if best is None else min(best, dt)
    if "-v" in sys.argv:
        print("   reps", lanes, sink_kind, piece, strict, all_, flush=True)
    return round(n / GIB / best, 2)


for lanes in (None, [0], [0, 0], [0, 0, 0], [0]):
    print("lanes", lanes, "count", run(lanes, "count", 64 * MIB),
          "store", run(lanes, "store", 64 * MIB), flush=True)
print("32K pipelined", run(None, "store", 32 << 10), "strict", run(None, "store", 32 << 10, True),
      flush=True)
print("1M pipelined", run(None, "store", MIB), "strict", run(None, "store", MIB, True), flush=True)

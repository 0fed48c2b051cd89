"""Per-call latency of the drop-in's one-blob calls (a Go glfs.PostBlob is one
Writer: glfsx_create with a store sink), single thread and with T threads
calling concurrently (each thread its own writers), plus glfsx_post_blobs
for the same blobs in one call.  Prints one JSON line.
usage: python scripts/latency.py [--threads 8] [--calls 400]"""
import ctypes
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    threads = int(sys.argv[sys.argv.index("--threads") + 1]) if "--threads" in sys.argv else 8
    calls = int(sys.argv[sys.argv.index("--calls") + 1]) if "--calls" in sys.argv else 400
    import numpy as np
    from glfs_amd import _native as N, glfs
    N.set_device(0)
    salt = glfs.Machine().make_salt("blob")
    sink = ctypes.cast(N.lib.glfsx_sink_count, N.POST_FN)
    bs = 2 << 20
    out = {}
    for size in (0, 9, 4096, 65536, 1 << 20, (2 << 20) + 1):
        data = np.frombuffer(os.urandom(max(size, 1)), dtype=np.uint8)

        def one(counts, root):
            N.check(N.lib.glfsx_create(bs, bs, salt, None, data.ctypes.data, size, sink,
                                       ctypes.byref(counts), ctypes.byref(root)))

        counts, root = (ctypes.c_uint64 * 2)(), N.glfsx_root()
        for _ in range(20):
            one(counts, root)
        ts = []
        for _ in range(calls):
            t = time.perf_counter()
            one(counts, root)
            ts.append(time.perf_counter() - t)
        ts.sort()

        def worker(n, res):
            c, r = (ctypes.c_uint64 * 2)(), N.glfsx_root()
            N.check(N.lib.glfsx_set_device(0))
            for _ in range(5):
                one(c, r)
            t = time.perf_counter()
            for _ in range(n):
                one(c, r)
            res.append(time.perf_counter() - t)

        res = []
        th = [threading.Thread(target=worker, args=(calls, res)) for _ in range(threads)]
        t0 = time.perf_counter()
        [t.start() for t in th]
        [t.join() for t in th]
        wall = time.perf_counter() - t0
        out[str(size)] = {"p50_us": round(ts[len(ts) // 2] * 1e6, 1),
                          "p90_us": round(ts[int(len(ts) * 0.9)] * 1e6, 1),
                          "calls_per_s_1_thread": round(1 / (sum(ts) / len(ts))),
                          f"calls_per_s_{threads}_threads": round(threads * calls / wall)}
    # the same 4 KiB blobs batched into one glfsx_post_blobs call
    n, ln = 4096, 4096
    blob = np.frombuffer(os.urandom(n * ln), dtype=np.uint8)
    offs = (ctypes.c_uint64 * n)(*[i * ln for i in range(n)])
    lens = (ctypes.c_uint64 * n)(*([ln] * n))
    roots = ctypes.create_string_buffer(64 * n)
    counts = (ctypes.c_uint64 * 2)()
    for _ in range(3):
        N.check(N.lib.glfsx_post_blobs(bs, bs, salt, None, blob.ctypes.data, offs, lens, n,
                                       sink, ctypes.byref(counts), roots))
    t = time.perf_counter()
    reps = 20
    for _ in range(reps):
        N.check(N.lib.glfsx_post_blobs(bs, bs, salt, None, blob.ctypes.data, offs, lens, n,
                                       sink, ctypes.byref(counts), roots))
    dt = (time.perf_counter() - t) / reps
    out["post_blobs_4096x4KiB"] = {"ms": round(dt * 1e3, 3), "blobs_per_s": round(n / dt)}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()

"""Secondary legs alone, for per-kernel profiling (rocprofv3 PMC passes):
config 4's small-blob kernels (bench.small_blobs) and the read side
(batched getF decrypt over a --gib GiB blob at 1 MiB blocks), and config 4
end to end (bench.config4_end_to_end: blobs, tree lines, tree blob).
usage: python scripts/legs.py [small|read|both|config4|config4one|config4all|postblob|config2|concat]
       [--gib G]"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def main():
    what = sys.argv[1] if len(sys.argv) > 1 else "both"
    gib = float(sys.argv[sys.argv.index("--gib") + 1]) if "--gib" in sys.argv else 16
    import torch
    from glfs_amd import _native as N
    torch.cuda.set_device(0)
    N.set_device(0)
    stream = torch.cuda.Stream()
    sp = ctypes.c_void_p(stream.cuda_stream)
    out = {}
    if what in ("small", "both"):
        out["small_blobs"] = bench.small_blobs(torch, N, stream, sp)
    if what in ("read", "both"):
        bs = bench.MIB
        per = int(gib * bench.GIB) // bs * bs
        with torch.cuda.stream(stream):
            data = torch.empty(per, dtype=torch.uint8, device="cuda")
            ct = torch.empty(per, dtype=torch.uint8, device="cuda")
            N.check(N.lib.glfsx_fill_splitmix_device(data.data_ptr(), 0, per, 3, sp))
        stream.synchronize()
        roof, _ = bench.roofline(torch, N, data, ct, per, bs, stream, sp)
        out["read_side"] = roof["read_side"]
    if what == "config4":
        out["config4_end_to_end"] = bench.config4_end_to_end(torch, N, stream, sp)
    if what == "config4one":   # the one-call route alone, 20 reps
        out["config4_one_call"] = bench.config4_end_to_end(torch, N, stream, sp, reps=20,
                                                           routes=("one_call",))
    if what == "config4all":   # all three routes, as the bench line
        out["config4_end_to_end"] = bench.config4_end_to_end(torch, N, stream, sp)
    if what == "postblob":     # per-call latency and concurrent callers
        out["postblob_latency"] = bench.postblob_latency(N)
        out["postblob_concurrency"] = bench.postblob_concurrency(N)
    if what == "config2":
        out["config2"] = bench.config2_leg(torch, N, stream, sp)
    if what == "concat":       # Concat from a native store (the GLFSX_CONCAT_TRACE build: timeline)
        out["concat"] = bench.concat_leg(N)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()

"""Config 2 (1 GiB at 2 MiB, bench.config2_leg) under split targets 1024 /
2048 / 4096 workgroups per pass (glfsx_set_split_target: G4 s1, G2 s2 -- the
default -- and G1 s3 items of k_pass_dc), interleaved, `reps` rounds.
usage: python scripts/c2_sweep.py [reps]  -> one JSON line"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    import torch
    from glfs_amd import _native as N
    torch.cuda.set_device(0)
    N.set_device(0)
    stream = torch.cuda.Stream()
    sp = ctypes.c_void_p(stream.cuda_stream)
    out = {}
    for _ in range(reps):
        for tgt in (1024, 2048, 4096):
            prev = N.lib.glfsx_set_split_target(tgt)
            r = bench.config2_leg(torch, N, stream, sp, steps=30, warmup=3)
            N.lib.glfsx_set_split_target(prev)
            out.setdefault(str(tgt), []).append(r["value"])
            out.setdefault("root_" + str(tgt), set()).add(r["root_cid"])
    for k in list(out):
        if k.startswith("root_"):
            out[k] = sorted(out[k])
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()

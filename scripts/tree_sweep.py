"""Config 4's tree blob under other latency-form plans (round 6).

The tree blob (115 blocks of 2 MiB) runs its DEK pass and the BLAKE3 pass
over its ctext at G4 s1 (230 workgroups, ~1 wave per SIMD), where rocprofv3
counters show each wave issuing one VALU instruction per ~4.9 cycles --
the one-wave issue rate of tools/chainlat.hip.  glfsx_set_latency_wgs moves
pass_plan's latency bound (5/8 of it), so the same Create runs at G2 s2
(460 workgroups) or G1 s3 (920), still in the latency form (two passes,
keystream launch + BLAKE3 pass): does a second or fourth wave per SIMD buy
issue slots here?  Per setting: the Create alone (HIP events, interleaved
reps, roots compared) and config 4 end to end (bench.config4_end_to_end,
the one-call route).
usage: python scripts/tree_sweep.py [reps] -> one JSON line"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402

MIB = 1 << 20


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    import torch
    from glfs_amd import _native as N
    torch.cuda.set_device(0)
    N.set_device(0)
    stream = torch.cuda.Stream()
    sp = ctypes.c_void_p(stream.cuda_stream)
    size, bs = 114 * 2 * MIB + 1234567, 2 * MIB   # 115 blocks, the last partial
    data = torch.empty(size, dtype=torch.uint8, device="cuda")
    ct = torch.empty(size, dtype=torch.uint8, device="cuda")
    N.check(N.lib.glfsx_fill_splitmix_device(data.data_ptr(), 0, size, 44, sp))
    stream.synchronize()
    root, posts = N.glfsx_root(), ctypes.c_uint64()
    out = {"tree_blob_bytes": size, "create_ms": {}, "config4_GiBps": {}, "roots": {}}
    settings = tuple(int(x) for x in os.environ.get("TREE_LW", "512,1024,2048").split(","))

    def create_ms(n=20):
        for _ in range(3):
            N.check(N.lib.glfsx_create_device(bs, None, None, data.data_ptr(), size,
                                              ct.data_ptr(), ctypes.byref(root),
                                              ctypes.byref(posts), sp))
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(n):
            N.check(N.lib.glfsx_create_device(bs, None, None, data.data_ptr(), size,
                                              ct.data_ptr(), ctypes.byref(root),
                                              ctypes.byref(posts), sp))
        e1.record(stream)
        e1.synchronize()
        return e0.elapsed_time(e1) / n

    for _ in range(reps):
        for lw in settings:
            prev = N.lib.glfsx_set_latency_wgs(lw)
            ms = create_ms()
            out["create_ms"].setdefault(str(lw), []).append(round(ms, 4))
            out["roots"].setdefault(str(lw), set()).add(bytes(root.ref)[:32].hex())
            r = bench.config4_end_to_end(torch, N, stream, sp, reps=10,
                                         routes=("device", "one_call"))
            out["config4_GiBps"].setdefault(str(lw), []).append(r["one_call"]["value"])
            out.setdefault("device_tree_create_ms", {}).setdefault(str(lw), []).append(
                r["device"]["pieces_ms"]["tree_create"])
            out.setdefault("c4_roots", {}).setdefault(str(lw), set()).add(
                r["one_call"]["tree_root_cid"])
            N.lib.glfsx_set_latency_wgs(prev)
    for key in ("roots", "c4_roots"):
        out[key] = {k: sorted(v) for k, v in out[key].items()}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()

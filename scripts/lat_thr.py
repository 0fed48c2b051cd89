"""Latency-mode threshold A/B (glfsx_set_latency_wgs) for a device-resident
Create: python scripts/lat_thr.py SIZE_MIB BS_KIB thr1 thr2 ... -> GiB/s per
threshold, interleaved over 3 reps (HIP events around 20 Creates)."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    size = int(sys.argv[1]) << 20
    bs = int(sys.argv[2]) << 10
    thrs = [int(x) for x in sys.argv[3:]]
    import torch
    from glfs_amd import _native as N
    torch.cuda.set_device(0)
    N.set_device(0)
    s = torch.cuda.current_stream()
    data = torch.empty(size, dtype=torch.uint8, device="cuda")
    ct = torch.empty(size, dtype=torch.uint8, device="cuda")
    N.check(N.lib.glfsx_fill_splitmix_device(data.data_ptr(), 0, size, 3, None))
    root = N.glfsx_root()
    out = {t: [] for t in thrs}
    roots = set()
    for _ in range(3):
        for t in thrs:
            N.set_latency_wgs(t)
            for _ in range(3):
                N.check(N.lib.glfsx_create_device(bs, None, None, data.data_ptr(), size,
                                                  ct.data_ptr(), ctypes.byref(root), None, None))
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for _ in range(20):
                N.check(N.lib.glfsx_create_device(bs, None, None, data.data_ptr(), size,
                                                  ct.data_ptr(), ctypes.byref(root), None, None))
            e1.record(s)
            e1.synchronize()
            out[t].append(round(20 * size / (1 << 30) / (e0.elapsed_time(e1) * 1e-3), 1))
            roots.add(bytes(root.ref))
    print(json.dumps({"size_mib": size >> 20, "bs_kib": bs >> 10, "gibs": out,
                      "one_root": len(roots) == 1}))


if __name__ == "__main__":
    main()

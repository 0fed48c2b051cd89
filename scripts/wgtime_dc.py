"""Tail of a fused split-mode launch (k_pass_dc), from the GLFSX_WGTIME build
(bash tools/build_variant.sh wgtime "-DGLFSX_WGTIME=1").  Runs
glfsx_create_device over SIZE GiB at block size BS a few times, reads the last
run's per-item timestamps (s_memrealtime, 100 MHz: DEK items at [0, 4096),
CID items at [4096, 8192)) and prints, over the whole launch:
  - span, and per-CU last item end (p0/p10/p50/p90/p100): how long CUs sit
    idle while the last items finish;
  - idle fraction of CU-time after each CU's last item ends;
  - item durations by kind (p0/p50/p90/p100) and the start time of the last
    items handed out.
usage: GLFSX_LIB=glfs_amd/libglfsx_wgtime.so python scripts/wgtime_dc.py [gib] [bs]"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch
    from glfs_amd import _native as N
    gib = float(sys.argv[1]) if len(sys.argv) > 1 else 1.0
    bs = int(sys.argv[2]) if len(sys.argv) > 2 else 2 << 20
    size = int(gib * (1 << 30))
    N.set_device(0)
    fn = N.lib.glfsx_debug_wgtime
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_void_p]
    s = torch.cuda.Stream()
    sp = ctypes.c_void_p(s.cuda_stream)
    data = torch.empty(size, dtype=torch.uint8, device="cuda")
    ct = torch.empty(size, dtype=torch.uint8, device="cuda")
    N.check(N.lib.glfsx_fill_splitmix_device(data.data_ptr(), 0, size, 7, sp))
    s.synchronize()
    root, n_posts = N.glfsx_root(), ctypes.c_uint64()
    res = []
    for rep in range(8):
        N.check(N.lib.glfsx_create_device(bs, None, None, data.data_ptr(), size, ct.data_ptr(),
                                          ctypes.byref(root), ctypes.byref(n_posts), sp))
        s.synchronize()
        if rep < 5:
            continue
        buf = np.zeros((8192, 8), dtype=np.uint64)
        N.check(fn(buf.ctypes.data))
        rows, kind = [], []
        for k, base in ((0, 0), (1, 4096)):
            r = buf[base:base + 4096]
            r = r[r[:, 0] > 0]
            rows.append(r)
            kind += [k] * len(r)
        r = np.concatenate(rows)
        kind = np.array(kind)
        t = r[:, :4].astype(np.int64)
        t0 = t[:, 0].min()
        start = (t[:, 0] - t0) / 100.0
        end = (t[:, 3] - t0) / 100.0
        hw = r[:, 4].astype(np.int64)
        xcc = r[:, 5].astype(np.int64) & 0xF
        cu_id = xcc * 256 + ((hw >> 13) & 7) * 32 + ((hw >> 12) & 1) * 16 + ((hw >> 8) & 0xF)
        span = float(end.max())
        cu_end = {}
        for c, e in zip(cu_id.tolist(), end.tolist()):
            cu_end[c] = max(cu_end.get(c, 0.0), e)
        ce = np.array(sorted(cu_end.values()))
        q = lambda a, ps=(0, 10, 50, 90, 100): [round(float(np.percentile(a, p)), 1) for p in ps]
        dur = end - start
        res.append({
            "items": int(len(r)), "dek_items": int((kind == 0).sum()),
            "cid_items": int((kind == 1).sum()), "cus": len(cu_end),
            "span_us": round(span, 1),
            "cu_last_end_us_p0_10_50_90_100": q(ce),
            "idle_after_cu_end_frac": round(float((span - ce).sum() / (len(ce) * span)), 4),
            "dek_item_us_p0_50_90_100": q(dur[kind == 0], (0, 50, 90, 100)),
            "cid_item_us_p0_50_90_100": q(dur[kind == 1], (0, 50, 90, 100)),
            "last_start_us": round(float(start.max()), 1),
        })
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()

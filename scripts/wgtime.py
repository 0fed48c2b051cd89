"""Phase timeline of the bulk passes' workgroups (diagnostics; needs the
GLFSX_WGTIME build: bash tools/build_variant.sh wgtime "-DGLFSX_WGTIME=1").
Runs glfsx_create_device over SIZE bytes at block size BS a few times, then
reads the last run's per-workgroup timestamps (s_memrealtime, 100 MHz) and
prints, per pass: span, start spread (rounds), chunk / subtree / merge phase
times, and how the first round's workgroups spread over XCDs and CUs.
usage: GLFSX_LIB=glfs_amd/libglfsx_wgtime.so python scripts/wgtime.py [gib] [bs]"""
import collections
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
    if os.environ.get("WG_LATENCY"):  # pass_plan's latency bound (glfsx_set_latency_wgs)
        N.lib.glfsx_set_latency_wgs(int(os.environ["WG_LATENCY"]))
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
    for _ in range(6):
        N.check(N.lib.glfsx_create_device(bs, None, None, data.data_ptr(), size, ct.data_ptr(),
                                          ctypes.byref(root), ctypes.byref(n_posts), sp))
    s.synchronize()
    buf = np.zeros((8192, 16), dtype=np.uint64)
    N.check(fn(buf.ctypes.data))
    out = {}
    for name, base in (("dek", 0), ("cid", 4096)):
        rows = buf[base:base + 4096]
        rows = rows[rows[:, 0] > 0]
        if len(rows) == 0:
            continue
        t = rows[:, :4].astype(np.int64)
        t0 = t[:, 0].min()
        rel = (t - t0) / 100.0  # us
        start, c_done, s_done, end = rel[:, 0], rel[:, 1], rel[:, 2], rel[:, 3]
        order = np.sort(start)
        # a gap of > 5 us between consecutive start times separates rounds
        gaps = np.where(np.diff(order) > 5.0)[0]
        r1 = int(gaps[0] + 1) if len(gaps) else len(order)
        hw = rows[:, 4].astype(np.int64)
        xcc = rows[:, 5].astype(np.int64) & 0xF
        cu = (hw >> 8) & 0xF
        sh = (hw >> 12) & 1
        se = (hw >> 13) & 0x7
        first = start < (order[r1 - 1] + 0.01)
        per_cu = collections.Counter(zip(xcc[first], se[first], sh[first], cu[first]))
        per_xcc = collections.Counter(xcc[first].tolist())
        q = lambda a: [round(float(np.percentile(a, p)), 1) for p in (0, 50, 90, 100)]
        out[name] = {
            "wgs": int(len(rows)),
            "span_us": round(float(end.max()), 1),
            "first_round_wgs": r1,
            "first_round_start_spread_us": round(float(order[r1 - 1]), 1),
            "second_round_start_us_p0_50_100": q(order[r1:]) if r1 < len(order) else None,
            "chunks_us_p0_50_90_100": q(c_done - start),
            "subtree_us_p0_50_90_100": q(s_done - c_done),
            "after_subtree_us_p0_50_90_100": q(end - s_done),
            "end_us_p0_50_90_100": q(end),
            "first_round_per_xcc": dict(sorted(per_xcc.items())),
            "first_round_cus": len(per_cu),
            "first_round_wgs_per_cu_hist": dict(sorted(collections.Counter(per_cu.values()).items())),
        }
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()

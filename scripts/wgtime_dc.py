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
        buf = np.zeros((8192, 16), dtype=np.uint64)
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
        # whole-message items (no split) return after their subtree (slot 2)
        last = np.where(t[:, 3] > 0, t[:, 3], np.where(t[:, 2] > 0, t[:, 2], t[:, 1]))
        end = (last - t0) / 100.0
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
        entry = np.where(r[:, 6] > 0, (r[:, 6].astype(np.int64) - t0) / 100.0, start)
        fetched = np.where(r[:, 7] > 0, (r[:, 7].astype(np.int64) - t0) / 100.0, start)
        pre = start - entry
        fetch = fetched - entry
        occ_entry = float((end - entry).sum() / span)
        # publish of the subtree CV + the arrival atomic (split items: slot 3 - slot 2)
        sp_ok = (t[:, 3] > 0) & (t[:, 2] > 0)
        arrive = (t[:, 3] - t[:, 2])[sp_ok] / 100.0
        chunks = (t[:, 1] - t[:, 0]) / 100.0
        subtree = ((t[:, 2] - t[:, 1]) / 100.0)[t[:, 2] > 0]
        ev = sorted([(x, 1) for x in start.tolist()] + [(x, -1) for x in end.tolist()])
        cur, peak, area, last = 0, 0, 0.0, 0.0
        for x, d in ev:
            area += cur * (x - last)
            last = x
            cur += d
            peak = max(peak, cur)
        bins = 24
        conc = [0.0] * bins
        for a0, b0 in zip(start.tolist(), end.tolist()):
            for k in range(bins):
                lo, hi = span * k / bins, span * (k + 1) / bins
                conc[k] += max(0.0, min(b0, hi) - max(a0, lo)) / (span / bins)
        per_cu_peak = {}
        for c in set(cu_id.tolist()):
            m = cu_id == c
            e2 = sorted([(x, 1) for x in start[m].tolist()] + [(x, -1) for x in end[m].tolist()])
            k = pk = 0
            for _, d in e2:
                k += d
                pk = max(pk, k)
            per_cu_peak[pk] = per_cu_peak.get(pk, 0) + 1
        by_kind = {}
        for kk, nm in ((0, "dek"), (1, "cid")):
            m = kind == kk
            if not m.any():
                continue
            s0, e0 = start[m], end[m]
            t1, ks = s0.min(), e0.max() - s0.min()
            cb = [0.0] * bins
            for a0, b0 in zip((s0 - t1).tolist(), (e0 - t1).tolist()):
                for k in range(bins):
                    lo, hi = ks * k / bins, ks * (k + 1) / bins
                    cb[k] += max(0.0, min(b0, hi) - max(a0, lo)) / (ks / bins)
            by_kind[nm] = {"span_us": round(float(ks), 1),
                           "mean_concurrent": round(float((e0 - s0).sum() / ks), 1),
                           "bins": [round(c) for c in cb]}
        res.append({
            "by_kind": by_kind,
            "entry_to_body_us_p0_50_90_100": q(pre, (0, 50, 90, 100)),
            "mean_concurrent_from_entry": round(occ_entry, 1),
            "entry_to_fetched_us_p0_50_90_100": q(fetch, (0, 50, 90, 100)),
            "fetch_us_median_by_entry_bin": [
                round(float(np.median(fetch[(entry >= span * k / 12) & (entry < span * (k + 1) / 12)])), 1)
                if ((entry >= span * k / 12) & (entry < span * (k + 1) / 12)).any() else None
                for k in range(12)],
            "fetch_us_median_dek_cid": [round(float(np.median(fetch[kind == 0])), 1),
                                        round(float(np.median(fetch[kind == 1])), 1)],
            "chunks_us_p0_50_90_100": q(chunks, (0, 50, 90, 100)),
            "subtree_merge_us_p0_50_90_100": q(subtree, (0, 50, 90, 100)),
            "publish_and_arrive_us_p0_50_90_100": q(arrive, (0, 50, 90, 100)),
            "items": int(len(r)), "dek_items": int((kind == 0).sum()),
            "cid_items": int((kind == 1).sum()), "cus": len(cu_end),
            "span_us": round(span, 1),
            "cu_last_end_us_p0_10_50_90_100": q(ce),
            "idle_after_cu_end_frac": round(float((span - ce).sum() / (len(ce) * span)), 4),
            "dek_item_us_p0_50_90_100": q(dur[kind == 0], (0, 50, 90, 100)),
            "cid_item_us_p0_50_90_100": q(dur[kind == 1], (0, 50, 90, 100)),
            "last_start_us": round(float(start.max()), 1),
            "peak_concurrent_items": peak,
            "mean_concurrent_items": round(area / span, 1),
            "cus_by_peak_items": dict(sorted(per_cu_peak.items())),
            "concurrency_by_time_bin": [round(c) for c in conc],
            "item_time_sum_over_slots_us": round(float(dur.sum()) / max(peak, 1), 1),
        })
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()

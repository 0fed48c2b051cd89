"""Where config 2's one-launch split post loses time against the headline's
per-byte rate, from the GLFSX_WGTIME build
(bash tools/build_variant.sh wgtime "-DGLFSX_WGTIME=1"; run with
GLFSX_LIB=glfs_amd/libglfsx_wgtime.so).

Config 2 = glfsx_create_device over 1 GiB at 2 MiB blocks: one k_pass_dc<2>
launch (2048 DEK items, 1536 coarse + 1024 fine CID items) plus the index
node.  Its slot-time (workgroup slots x the launch's span, slots = 4 per CU)
is split into:
  ramp     idle slot-time before the slots first fill;
  prologue each item's kernel entry -> its body start (item fetch, waiting
           for issue behind the resident waves);
  dek_wait a CID item's wait for its message's DEK (k_pass_dc's s_sleep loop);
  body     the rest of each item (chunks, subtree merge, publish);
  drain    idle slot-time after the slots stop being refilled.
Each term / slots = its share of the launch in us.  The headline's rate is
measured the same way on a 4 GiB blob at 1 MiB blocks (its two k_pass launches,
4096 workgroups each, the headline's kernels): body us per GiB per slot.
usage: GLFSX_LIB=... python scripts/c2_attrib.py [reps]  -> one JSON line"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
GIB, MIB = 1 << 30, 1 << 20


def stamps(N, fn):
    import numpy as np
    buf = np.zeros((8192, 16), dtype=np.uint64)
    N.check(fn(buf.ctypes.data))
    return buf


def rows(buf, base):
    import numpy as np
    r = buf[base:base + 4096]
    return r[r[:, 0] > 0].astype(np.int64)


def item_times(r):
    """(entry, start, wait_end, end) in ticks for each item row."""
    import numpy as np
    start = r[:, 0]
    end = np.where(r[:, 3] > 0, r[:, 3], np.where(r[:, 2] > 0, r[:, 2], r[:, 1]))
    # slots 6 / 8 are only stamped by k_pass_dc: stale values of an earlier
    # launch (k_pass leaves them alone) fall outside [start - 1 ms, end]
    ok6 = (r[:, 6] > 0) & (r[:, 6] <= start) & (start - r[:, 6] < 100000)
    ok8 = (r[:, 8] >= start) & (r[:, 8] <= end)
    entry = np.where(ok6, r[:, 6], start)
    wait_end = np.where(ok8, r[:, 8], start)
    return entry, start, wait_end, end


def cu_ids(r):
    import numpy as np
    hw = r[:, 4]
    xcc = r[:, 5] & 0xF
    return xcc * 256 + ((hw >> 13) & 7) * 32 + ((hw >> 12) & 1) * 16 + ((hw >> 8) & 0xF)


def attrib(r):
    import numpy as np
    entry, start, wait_end, end = item_times(r)
    t0 = entry.min()
    span = (end.max() - t0) / 100.0
    cus = len(set(cu_ids(r).tolist()))
    slots = 4 * cus
    e = (entry - t0) / 100.0
    s = (start - t0) / 100.0
    w = (wait_end - t0) / 100.0
    f = (end - t0) / 100.0
    # occupancy curve (items from entry to end)
    ev = sorted([(x, 1) for x in e.tolist()] + [(x, -1) for x in f.tolist()])
    cur, area_ramp, last, t_full = 0, 0.0, 0.0, None
    for x, d in ev:
        if t_full is None:
            area_ramp += (slots - cur) * (x - last)
        last = x
        cur += d
        if t_full is None and cur >= 0.97 * slots:
            t_full = x
    t_full = t_full if t_full is not None else 0.0
    t_last_entry = float(e.max())
    busy = float((f - e).sum())
    idle = slots * span - busy
    # drain: idle slot-time after the last item entered
    in_drain = 0.0
    for a0, b0 in zip(e.tolist(), f.tolist()):
        in_drain += max(0.0, b0 - max(a0, t_last_entry))
    drain = slots * (span - t_last_entry) - in_drain
    prologue = float((s - e).sum())
    dek_wait = float((w - s).sum())
    body = float((f - w).sum())
    other_idle = idle - area_ramp - drain
    per = lambda x: round(x / slots, 1)
    return {"span_us": round(span, 1), "slots": slots, "items": int(len(r)),
            "t_full_us": round(t_full, 1), "last_entry_us": round(t_last_entry, 1),
            "us_of_launch": {"ramp": per(area_ramp), "prologue": per(prologue),
                             "dek_wait": per(dek_wait), "body": per(body),
                             "drain": per(drain), "other_idle": per(other_idle)},
            "dek_wait_items_over_1us": int(((w - s) > 1.0).sum()),
            "dek_wait_us_p50_90_100": [round(float(np.percentile(w - s, p)), 2)
                                       for p in (50, 90, 100)]}


def main():
    import numpy as np
    import torch
    from glfs_amd import _native as N
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    N.set_device(0)
    fn = N.lib.glfsx_debug_wgtime
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_void_p]
    st = torch.cuda.Stream()
    sp = ctypes.c_void_p(st.cuda_stream)
    out = {"config2": [], "headline_4gib": []}
    root, n_posts = N.glfsx_root(), ctypes.c_uint64()
    # config 2
    size, bs = GIB, 2 * MIB
    data = torch.empty(size, dtype=torch.uint8, device="cuda")
    ct = torch.empty(size, dtype=torch.uint8, device="cuda")
    N.check(N.lib.glfsx_fill_splitmix_device(data.data_ptr(), 0, size, 1, sp))
    st.synchronize()
    for rep in range(3 + reps):
        N.check(N.lib.glfsx_create_device(bs, None, None, data.data_ptr(), size, ct.data_ptr(),
                                          ctypes.byref(root), ctypes.byref(n_posts), sp))
        st.synchronize()
        if rep < 3:
            continue
        buf = stamps(N, fn)
        r = np.concatenate([rows(buf, 0), rows(buf, 4096)])
        a = attrib(r)
        a["body_us_per_gib_per_slot"] = round(a["us_of_launch"]["body"] * GIB / size, 1)
        out["config2"].append(a)
    del data, ct
    torch.cuda.empty_cache()
    # the headline's kernels: 4 GiB at 1 MiB = 4096 workgroups per pass
    size, bs = 4 * GIB, MIB
    data = torch.empty(size, dtype=torch.uint8, device="cuda")
    ct = torch.empty(size, dtype=torch.uint8, device="cuda")
    N.check(N.lib.glfsx_fill_splitmix_device(data.data_ptr(), 0, size, 3, sp))
    st.synchronize()
    for rep in range(2 + reps):
        N.check(N.lib.glfsx_create_device(bs, None, None, data.data_ptr(), size, ct.data_ptr(),
                                          ctypes.byref(root), ctypes.byref(n_posts), sp))
        st.synchronize()
        if rep < 2:
            continue
        buf = stamps(N, fn)
        h = {}
        for nm, base in (("dek", 0), ("cid", 4096)):
            a = attrib(rows(buf, base))
            a["body_us_per_gib_per_slot"] = round(a["us_of_launch"]["body"] * GIB / size, 1)
            h[nm] = a
        out["headline_4gib"].append(h)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()

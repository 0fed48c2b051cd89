"""Where a one-shot PostBlob's time goes: `calls` back-to-back glfsx_create
of one blob size from one thread, then (run under rocprofv3 --kernel-trace)
the kernel's own duration against the call's wall time.

  rocprofv3 --kernel-trace -f csv -d OUT -o run -- python scripts/one_trace.py SIZE
  python scripts/one_trace.py --report OUT SIZE
"""
import csv
import ctypes
import glob
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run(size, calls=400):
    import numpy as np
    from glfs_amd import _native as N
    from glfs_amd import glfs
    salt = glfs.Machine().make_salt("blob")
    sink = ctypes.cast(N.lib.glfsx_sink_count, N.POST_FN)
    counts, root = (ctypes.c_uint64 * 2)(), N.glfsx_root()
    data = np.frombuffer(np.random.default_rng(size).bytes(max(size, 1)), dtype=np.uint8)
    ts = []
    timing = getattr(N.lib, "glfsx_debug_one_timing", None)   # GLFSX_ONE_TIMING builds
    tv = (ctypes.c_uint64 * 16)()
    for i in range(calls + 20):
        if i == 20 and timing:
            timing(1, tv)
        t = time.perf_counter()
        N.check(N.lib.glfsx_create(2 << 20, 2 << 20, salt, None, data.ctypes.data, size,
                                   sink, ctypes.byref(counts), ctypes.byref(root)))
        if i >= 20:
            ts.append(time.perf_counter() - t)
    ts.sort()
    out = {"size": size, "calls": calls, "p50_us": round(ts[len(ts) // 2] * 1e6, 1),
           "p10_us": round(ts[len(ts) // 10] * 1e6, 1)}
    if timing:
        timing(0, tv)
        k = max(tv[15], 1)
        out["k_one_phase_end_us"] = dict(zip(
            ("read_desc", "stage", "dek", "keystream", "cid_ref", "signal",
             "dek_chunks", "cid_chunks"),
            (round(tv[i] / k / 100.0, 2) for i in range(8))))   # 100 MHz ticks
        out["timed_launches"] = tv[15]
        out["k_one_clock_GHz"] = round(tv[13] / max(tv[14], 1) * 0.1, 3)
    print(json.dumps(out))


def report(d, size):
    path = glob.glob(os.path.join(d, "**", "*_kernel_trace.csv"), recursive=True)[0]
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    ks = [r for r in rows if "k_one" in r["Kernel_Name"] or "k_med" in r["Kernel_Name"]]
    ks = ks[20:]
    dur = sorted((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in ks)
    gaps = sorted((int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1e3
                  for a, b in zip(ks, ks[1:]))
    pct = lambda v, q: v[int(len(v) * q)] if v else None
    print(json.dumps({"size": size, "kernels": len(ks),
                      "kernel_us": {"p10": pct(dur, .1), "p50": pct(dur, .5), "p90": pct(dur, .9)},
                      "end_to_next_start_us": {"p10": pct(gaps, .1), "p50": pct(gaps, .5),
                                               "p90": pct(gaps, .9)},
                      "names": sorted(set(r["Kernel_Name"].split("(")[0] for r in ks))}))


if __name__ == "__main__":
    if sys.argv[1] == "--report":
        report(sys.argv[2], int(sys.argv[3]))
    else:
        run(int(sys.argv[1]))

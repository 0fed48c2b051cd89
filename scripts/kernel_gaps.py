"""Per-step kernel timeline from a rocprofv3 kernel trace: the kernels of one
bigblob write (glfsx_create_device) in launch order, each with its duration
and the idle gap before it, plus the step's GPU-busy vs first-to-last span.
A step starts at each launch of the kernel named by `start` (default: the
runtime's fillBuffer kernel if the trace has one -- round 2's per-step
memset of the level-1 node buffer -- else the first non-fill kernel of the
trace, e.g. k_pass_dc for config 2 or k_small_q for config 4).

usage: python scripts/kernel_gaps.py <trace_dir_with_kernel_trace_csv> [skip] [start]
"""
import csv
import glob
import os
import sys


def short(name):
    name = name.replace("glfsx::(anonymous namespace)::", "")
    return name.split("(")[0].replace("void ", "")


def main(d, skip=3, start=None):
    path = glob.glob(os.path.join(d, "**", "*_kernel_trace.csv"), recursive=True)[0]
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    names = [short(r["Kernel_Name"]) for r in rows]
    if start is None:
        start = "fillBuffer" if any("fillBuffer" in k for k in names) else \
            next(k for k in names if not k.startswith("k_fill"))
    steps, cur = [], None
    for r in rows:
        k = short(r["Kernel_Name"])
        if k.startswith("k_fill"):
            continue
        if start in k:
            cur = []
            steps.append(cur)
        if cur is not None:
            cur.append((k, int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                        r.get("Grid_Size", r.get("Grid_Size_X"))))
    steps = [s for s in steps if len(s) > 1][skip:]
    if not steps:
        print("no steps found")
        return
    spans, busys = [], []
    for s in steps:
        spans.append(s[-1][2] - s[0][1])
        busys.append(sum(e - b for _, b, e, _ in s))
    print(f"{len(steps)} steps; kernels per step {len(steps[0])}; "
          f"span {sum(spans) / len(spans) / 1e3:.1f} us, busy {sum(busys) / len(busys) / 1e3:.1f} us, "
          f"idle {(sum(spans) - sum(busys)) / len(spans) / 1e3:.1f} us")
    s = steps[len(steps) // 2]
    prev = None
    for k, b, e, g in s:
        gap = (b - prev) / 1e3 if prev is not None else 0.0
        print(f"  {k:45s} grid={g:>9} {(e - b) / 1e3:9.1f} us   gap {gap:6.1f} us")
        prev = e


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 3,
         sys.argv[3] if len(sys.argv) > 3 else None)

"""Config-4 one-call timeline from a rocprofv3 kernel (+ memory copy) trace of
`scripts/legs.py config4one`: every kernel and copy of one call, both
streams, as start / end offsets from the call's first kernel (the blobs'
DEK pass, or k_tree_len where the layout goes first), plus the mean span
over the calls (warm-up calls skipped).

usage: python scripts/c4_timeline.py <trace dir> [skip]"""
import csv
import glob
import os
import sys


def short(name):
    name = name.replace("glfsx::(anonymous namespace)::", "")
    return name.split("(")[0].replace("void ", "")


def rows_of(d, pat):
    out = []
    for p in glob.glob(os.path.join(d, "**", pat), recursive=True):
        out += list(csv.DictReader(open(p)))
    return out


def main(d, skip=2):
    ev = []
    for r in rows_of(d, "*_kernel_trace.csv"):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]),
                   r.get("Queue_Id", "?")))
    for r in rows_of(d, "*_memory_copy_trace.csv"):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                   "copy " + r.get("Direction", "?"), "copy"))
    ev.sort()
    # a call starts with its blobs' DEK pass when that is queued first (the
    # default order), else with the layout
    names = [e[2] for e in ev]
    first = next((k for k in names if k.startswith("k_small_q<4, false") or k == "k_tree_len"),
                 "k_tree_len")
    calls, cur = [], None
    for e in ev:
        if e[2].startswith("k_fill"):
            continue
        if e[2] == first:
            cur = []
            calls.append(cur)
        if cur is not None:
            cur.append(e)
    calls = [c for c in calls if len(c) > 3][skip:]
    if not calls:
        print("no calls found")
        return
    spans = [max(e[1] for e in c) - c[0][0] for c in calls]
    print(f"{len(calls)} calls; span mean {sum(spans) / len(spans) / 1e3:.1f} us, "
          f"min {min(spans) / 1e3:.1f}, max {max(spans) / 1e3:.1f}")
    c = calls[len(calls) // 2]
    t0 = c[0][0]
    for b, e, k, q in c:
        print(f"  {k:42s} q={q:>4} start {(b - t0) / 1e3:8.1f}  end {(e - t0) / 1e3:8.1f}"
              f"  dur {(e - b) / 1e3:8.1f} us")
    if len(calls) > 1:
        gaps = [calls[i + 1][0][0] - max(e[1] for e in calls[i]) for i in range(len(calls) - 1)]
        print(f"between calls (end of one to the next call's first kernel): mean "
              f"{sum(gaps) / len(gaps) / 1e3:.1f} us")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 2)

"""Per-size median kernel durations from a quad_lat.py kernel trace
(rocprofv3 --kernel-trace): the k_fill markers separate the sizes.
usage: python scripts/quad_lat_sum.py <dir with *_kernel_trace.csv>"""
import collections
import csv
import glob
import json
import os
import sys

SIZES = [64, 1024, 16 << 10, 64 << 10, 256 << 10, 1 << 20, 2 << 20]


def short(n):
    n = n.replace("void ", "").replace("glfsx::(anonymous namespace)::", "")
    return n.split("(")[0]


def main(d):
    rows = list(csv.DictReader(open(glob.glob(os.path.join(d, "*kernel_trace.csv"))[0])))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    groups, cur = [], None
    for r in rows:
        n = short(r["Kernel_Name"])
        dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0
        if n == "k_fill":
            cur = collections.defaultdict(list)
            groups.append(cur)
        elif cur is not None:
            cur[n].append(dur)
    out = {}
    for sz, g in zip(SIZES, groups):
        out[sz] = {k: round(sorted(v)[len(v) // 2], 2) for k, v in g.items()}
    print(json.dumps(out))


if __name__ == "__main__":
    main(sys.argv[1])

"""Per (kernel, grid, workgroup) dispatch groups of a rocprofv3 kernel trace:
count, mean and total duration.  Distinguishes launches of one kernel under
different plans (scripts/tree_sweep.py under rocprofv3 --kernel-trace).
usage: python scripts/trace_groups.py kernel_trace.csv [name-substring ...]"""
import csv
import sys
from collections import defaultdict


def main():
    path, subs = sys.argv[1], sys.argv[2:]
    groups = defaultdict(list)
    with open(path) as f:
        for r in csv.DictReader(f):
            name = r["Kernel_Name"]
            if subs and not any(s in name for s in subs):
                continue
            grid = r.get("Grid_Size_X") or r.get("Grid_Size")
            wg = r.get("Workgroup_Size_X") or r.get("Workgroup_Size")
            dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            groups[(name[:60], grid, wg)].append(dur)
    rows = sorted(groups.items(), key=lambda kv: -sum(kv[1]))
    print("%-60s %9s %5s %6s %9s %10s" % ("kernel", "grid", "wg", "count", "mean_us", "total_us"))
    for (name, grid, wg), d in rows:
        print("%-60s %9s %5s %6d %9.1f %10.1f" % (name, grid, wg, len(d), sum(d) / len(d), sum(d)))


if __name__ == "__main__":
    main()

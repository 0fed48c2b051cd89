"""Summarise rocprofv3 CSV output (kernel trace + PMC passes) into a JSON file.

usage: python scripts/prof_summary.py <prof_dir> <out.json>
For every (kernel, grid) pair: dispatch count, mean duration (kernel trace),
and per-dispatch counter means.  FETCH_SIZE is reported both raw (KB, as
rocprofv3 gives it) and corrected x2 per MI355X_MICROARCH.md ("FETCH_SIZE
reports exactly 1/2 of the bytes of a wide coalesced streaming read").
"""
import collections
import csv
import glob
import json
import os
import sys


def short(name):
    name = name.replace("glfsx::(anonymous namespace)::", "")
    return name.split("(")[0].replace("void ", "")


def main(d, out):
    res = {}
    for path in glob.glob(os.path.join(d, "*", "*_kernel_trace.csv")):
        pas = os.path.basename(os.path.dirname(path))
        rows = list(csv.DictReader(open(path)))
        agg = collections.defaultdict(list)
        for r in rows:
            key = f"{short(r['Kernel_Name'])} grid={r.get('Grid_Size', r.get('Grid_Size_X'))}"
            agg[key].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
        for k, v in agg.items():
            e = res.setdefault(pas, {}).setdefault(k, {})
            e["dispatches"] = len(v)
            e["mean_ns"] = sum(v) / len(v)
            e["min_ns"] = min(v)
    for path in glob.glob(os.path.join(d, "*", "*_counter_collection.csv")):
        pas = os.path.basename(os.path.dirname(path))
        rows = list(csv.DictReader(open(path)))
        agg = collections.defaultdict(lambda: collections.defaultdict(list))
        for r in rows:
            key = f"{short(r['Kernel_Name'])} grid={r.get('Grid_Size', r.get('Grid_Size_X'))}"
            agg[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
            agg[key]["_dur_ns"].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
        for k, cs in agg.items():
            e = res.setdefault(pas, {}).setdefault(k, {})
            n = len(cs["_dur_ns"]) // max(1, len([c for c in cs if c != "_dur_ns"]))
            for c, v in cs.items():
                if c == "_dur_ns":
                    continue
                e[c] = sum(v) / len(v)
            durs = cs["_dur_ns"]
            e["pmc_mean_ns"] = sum(durs) / len(durs)
            if "FETCH_SIZE" in e:
                e["FETCH_bytes_corrected_x2"] = e["FETCH_SIZE"] * 1024 * 2
            if "WRITE_SIZE" in e:
                e["WRITE_bytes"] = e["WRITE_SIZE"] * 1024
            if "GRBM_GUI_ACTIVE" in e:
                e["eff_clock_GHz"] = e["GRBM_GUI_ACTIVE"] / 8 / e["pmc_mean_ns"]
    json.dump(res, open(out, "w"), indent=1, sort_keys=True)
    for pas, ks in sorted(res.items()):
        print("==", pas)
        for k, e in sorted(ks.items(), key=lambda kv: -kv[1].get("mean_ns", kv[1].get("pmc_mean_ns", 0))):
            print(" ", k, {kk: (round(vv, 3) if isinstance(vv, float) else vv) for kk, vv in e.items()})


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])

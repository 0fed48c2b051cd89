"""Derive per-launch HBM traffic for bench.py's roofline.traffic from a
prof_summary.py JSON (rocprofv3 PMC passes at 16 GiB, scaled to the 64 GiB
bench launch).  usage: python scripts/pmc_traffic.py profiles/r1/summary.json profiles/pmc_traffic.json
"""
import json
import sys

s = json.load(open(sys.argv[1]))


def g(pas, prefix):
    return [v for k, v in s[pas].items() if k.startswith(prefix) and "grid=4194304" in k][0]


n = 16 * 2**30          # bytes per launch in the PMC runs
scale = 4               # 64 GiB bench launch / 16 GiB PMC launch (linear in blocks)
dek_f, cid_f = g("fetch", "k_pass<4, false"), g("fetch", "k_pass<4, true")
cid_w = g("write", "k_pass<4, true")
cal = n / (dek_f["FETCH_SIZE"] * 1024)  # the DEK pass reads every input byte exactly once
rd = cid_f["FETCH_SIZE"] * 1024 * cal * scale
wr = cid_w["WRITE_SIZE"] * 1024 * scale
sq_d, sq_c = g("sq", "k_pass<4, false"), g("sq", "k_pass<4, true")
out = {
    "note": ("HBM bytes per launch from rocprofv3 PMC (separate passes, --kernel-trace only), "
             "16 GiB runs scaled x4 to the 64 GiB bench launch.  FETCH_SIZE is calibrated on "
             "this kernel family's own access pattern: the DEK pass reads each input byte "
             "exactly once, giving a factor %.3f (the guide's x2 is for wide coalesced "
             "streams).  WRITE_SIZE taken as-is." % cal),
    "fetch_calibration": cal,
    "dek": {"hbm_bytes_per_launch": n * scale, "read_bytes": n * scale, "write_bytes": 0,
            "algorithmic_bytes": n * scale},
    "cid": {"hbm_bytes_per_launch": int(rd + wr), "read_bytes": int(rd), "write_bytes": int(wr),
            "algorithmic_bytes": 2 * n * scale},
    "clock_GHz": {"dek": sq_d["eff_clock_GHz"], "cid": sq_c["eff_clock_GHz"]},
    "valu_instr_per_64B_block": {"dek": sq_d["SQ_INSTS_VALU"] / (n / 4096),
                                 "cid": sq_c["SQ_INSTS_VALU"] / (n / 4096)},
}
json.dump(out, open(sys.argv[2], "w"), indent=1)
print(json.dumps(out, indent=1))

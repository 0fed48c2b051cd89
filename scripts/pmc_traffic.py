"""Per-launch HBM traffic for bench.py's roofline.traffic, from a
prof_summary.py JSON of scripts/profile.sh's PMC passes (64 GiB launches, the
bench workload itself).

usage: python scripts/pmc_traffic.py profiles/r1/summary.json profiles/pmc_traffic.json

Corrections per MI355X_MICROARCH.md "HBM": both passes read plaintext with
buffer_load ... lds (16 B per lane, 8 full 128-B lines per instruction), the
wide coalesced streaming read for which FETCH_SIZE reports exactly half the
bytes, so FETCH_SIZE x 1024 x 2; the CID pass stores ctext with 16 B per lane,
8 full lines per instruction, for which WRITE_SIZE is exact.  Cross-check: the
DEK pass reads each plaintext byte exactly once, so its corrected FETCH must
come out at the launch's byte count ("dek_fetch_vs_bytes").
"""
import json
import sys

s = json.load(open(sys.argv[1]))
GRID = "grid=16777216"   # 65536 blocks x 256 lanes: the 64 GiB @ 1 MiB launch
n = 64 * 2**30


def g(pas, prefix):
    return [v for k, v in s[pas].items() if k.startswith(prefix) and GRID in k][0]


dek_f, cid_f = g("fetch", "k_pass<4, false"), g("fetch", "k_pass<4, true")
dek_w, cid_w = g("write", "k_pass<4, false"), g("write", "k_pass<4, true")
sq_d, sq_c = g("sq", "k_pass<4, false"), g("sq", "k_pass<4, true")
rd = lambda e: e["FETCH_SIZE"] * 1024 * 2
wr = lambda e: e["WRITE_SIZE"] * 1024
out = {
    "note": ("HBM bytes per 64 GiB launch from rocprofv3 PMC (separate passes, "
             "--kernel-trace only): FETCH_SIZE x2 (wide coalesced buffer_load...lds reads), "
             "WRITE_SIZE as-is (16-B-per-lane full-line stores); MI355X_MICROARCH.md HBM."),
    "dek_fetch_vs_bytes": rd(dek_f) / n,
    "dek": {"hbm_bytes_per_launch": int(rd(dek_f) + wr(dek_w)), "read_bytes": int(rd(dek_f)),
            "write_bytes": int(wr(dek_w)), "algorithmic_bytes": n},
    "cid": {"hbm_bytes_per_launch": int(rd(cid_f) + wr(cid_w)), "read_bytes": int(rd(cid_f)),
            "write_bytes": int(wr(cid_w)), "algorithmic_bytes": 2 * n},
    "clock_GHz": {"dek": sq_d["eff_clock_GHz"], "cid": sq_c["eff_clock_GHz"]},
    "valu_instr_per_64B_block": {"dek": sq_d["SQ_INSTS_VALU"] / (n / 4096),
                                 "cid": sq_c["SQ_INSTS_VALU"] / (n / 4096)},
}
json.dump(out, open(sys.argv[2], "w"), indent=1)
print(json.dumps(out, indent=1))

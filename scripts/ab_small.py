"""Config 4 A/B under environment settings, interleaved: small_blobs
(1M x 4 KiB hashing) and config4_end_to_end per setting, each in its own
process.  usage: python scripts/ab_small.py REPS "K=V ..." "K=V ..." ..."""
import json
import os
import statistics
import subprocess
import sys

reps, settings = int(sys.argv[1]), sys.argv[2:]
res = {s: {"small": [], "c4": []} for s in settings}
for r in range(reps):
    for st in settings:
        env = dict(os.environ)
        for kv in st.split():
            k, v = kv.split("=", 1)
            env[k] = v
        p = subprocess.run([sys.executable, "scripts/legs.py", "config4"], env=env,
                           capture_output=True, text=True, timeout=300)
        q = subprocess.run([sys.executable, "scripts/legs.py", "small"], env=env,
                           capture_output=True, text=True, timeout=300)
        try:
            c4 = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][0])
            sb = json.loads([ln for ln in q.stdout.splitlines() if ln.startswith("{")][0])
        except IndexError:
            print(st, "failed", p.stderr[-1500:], q.stderr[-1500:], flush=True)
            sys.exit(1)
        res[st]["small"].append(sb["small_blobs"]["value"])
        res[st]["c4"].append(c4["config4_end_to_end"]["value"])
        three = c4["config4_end_to_end"].get("three_calls", {})
        print(r, st, "small", res[st]["small"][-1], "c4 one_call", res[st]["c4"][-1],
              "three_calls", three.get("value"), three.get("pieces_ms"), flush=True)
for st, d in res.items():
    print(f"[{st}] small median {statistics.median(d['small']):.2f}  "
          f"config4 median {statistics.median(d['c4']):.2f}")

"""Interleaved A/B of environment settings on one bench configuration.
usage: python scripts/ab_envcfg.py REPS "bench args" "K=V ..." "K=V ..." ...
("-" for no extra setting).  Prints every run and, per setting, the median
and mean of `value`."""
import json
import os
import statistics
import subprocess
import sys

reps, cfg, settings = int(sys.argv[1]), sys.argv[2].split(), sys.argv[3:]
res = {st: [] for st in settings}
for r in range(reps):
    for st in settings:
        env = dict(os.environ)
        for kv in st.split():
            if kv != "-":
                k, v = kv.split("=", 1)
                env[k] = v
        p = subprocess.run([sys.executable, "bench.py", "--no-extras", *cfg], env=env,
                           capture_output=True, text=True, timeout=300)
        line = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
        if not line:
            print(st, "failed", p.stderr[-2000:], flush=True)
            sys.exit(1)
        v = json.loads(line[0])["value"]
        res[st].append(v)
        print(r, st, v, flush=True)
for st, v in res.items():
    print(f"[{st}] median {statistics.median(v):8.2f} mean {statistics.mean(v):8.2f} "
          f"min {min(v):8.2f} max {max(v):8.2f}")

"""A/B tuning runs: for each library build (GLFSX_LIB), the headline bench
(--no-extras) and the secondary legs, each in its own process, REPS rounds
interleaved; prints one summary line per library.
usage: python scripts/ab.py [--reps R] lib1.so lib2.so ..."""
import json
import os
import subprocess
import sys

args = sys.argv[1:]
reps = 2
if args and args[0] == "--reps":
    reps, args = int(args[1]), args[2:]
res = {lib: {"head": [], "small": [], "read": []} for lib in args}
for r in range(reps):
    for lib in args:
        env = dict(os.environ, GLFSX_LIB=lib)
        out = subprocess.run([sys.executable, "bench.py", "--no-extras", "--steps", "5"],
                             env=env, capture_output=True, text=True, timeout=300)
        line = [l for l in out.stdout.splitlines() if l.startswith("{")]
        if line:
            res[lib]["head"].append(json.loads(line[0])["value"])
        else:
            print(lib, "bench failed", out.stderr[-2000:], flush=True)
            sys.exit(1)
        out = subprocess.run([sys.executable, "scripts/legs.py"], env=env,
                             capture_output=True, text=True, timeout=300)
        line = [l for l in out.stdout.splitlines() if l.startswith("{")]
        if line:
            d = json.loads(line[0])
            res[lib]["small"].append(d["small_blobs"]["value"])
            res[lib]["read"].append(d["read_side"]["value"])
        else:
            print(lib, "legs failed", out.stderr[-2000:], flush=True)
            sys.exit(1)
        print(r, lib, res[lib]["head"][-1], res[lib]["small"][-1], res[lib]["read"][-1], flush=True)
for lib, d in res.items():
    print(f"{os.path.basename(lib):28s} head {max(d['head']):8.2f}  small {max(d['small']):8.2f}  "
          f"read {max(d['read']):8.2f}")

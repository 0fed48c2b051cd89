"""Interleaved A/B of library builds on one bench configuration.
usage: python scripts/ab_cfg.py REPS "bench args" lib1.so lib2.so ...
Prints every run and, per library, the median and mean of `value`."""
import json
import os
import statistics
import subprocess
import sys

reps, cfg, libs = int(sys.argv[1]), sys.argv[2].split(), sys.argv[3:]
res = {lib: [] for lib in libs}
for r in range(reps):
    for lib in libs:
        env = dict(os.environ, GLFSX_LIB=lib)
        p = subprocess.run([sys.executable, "bench.py", "--no-extras", *cfg], env=env,
                           capture_output=True, text=True, timeout=300)
        line = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
        if not line:
            print(lib, "failed", p.stderr[-2000:], flush=True)
            sys.exit(1)
        v = json.loads(line[0])["value"]
        res[lib].append(v)
        print(r, os.path.basename(lib), v, flush=True)
for lib, v in res.items():
    print(f"{os.path.basename(lib):24s} median {statistics.median(v):8.2f} mean "
          f"{statistics.mean(v):8.2f} min {min(v):8.2f} max {max(v):8.2f}")

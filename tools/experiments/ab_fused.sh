#!/bin/bash
# Config 2 (1 GiB at 2 MiB) and a 64 MiB blob: fused split-mode launch
# (default), its 3-waves register budget (libglfsx_fw1.so) and the two-launch
# form (GLFSX_FUSED=0), interleaved.  usage: bash scripts/ab_fused.sh [reps]
REPS=${1:-2}
for r in $(seq $REPS); do
  for v in "glfs_amd/libglfsx.so:1" "glfs_amd/libglfsx_fw1.so:1" "glfs_amd/libglfsx.so:0"; do
    lib=${v%%:*}; f=${v##*:}
    for cfg in "--size-gib 1 --block-size 2097152" "--size-gib 0.0625"; do
      x=$(GLFSX_LIB=$lib GLFSX_FUSED=$f timeout -k 10 120 python bench.py --no-extras $cfg --steps 50 --warmup 5 2>/dev/null | python -c "import json,sys; print(json.loads(sys.stdin.read())['value'])")
      echo "$r $(basename $lib) fused=$f $cfg $x"
    done
  done
done

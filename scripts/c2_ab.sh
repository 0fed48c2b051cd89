#!/bin/bash
# Config 2 (1 GiB at 2 MiB blocks, device-resident) and a 64 MiB blob, A/B
# of library builds x split targets, interleaved in one box session.
# usage: bash scripts/c2_ab.sh "lib1.so lib2.so" "2048 1024" [reps]
LIBS=$1; SPLITS=$2; REPS=${3:-2}
for r in $(seq $REPS); do for lib in $LIBS; do for sp in $SPLITS; do
  for cfg in "--size-gib 1 --block-size 2097152" "--size-gib 0.0625"; do
    v=$(GLFSX_LIB=$lib GLFSX_SPLIT_WG=$sp timeout -k 10 120 python bench.py --no-extras $cfg --steps 50 --warmup 5 | python -c "import json,sys; print(json.loads(sys.stdin.read())['value'])")
    echo "$r $(basename $lib) split=$sp $cfg $v"
  done
done; done; done

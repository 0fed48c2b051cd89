#!/bin/bash
# config-2 / 64 MiB A/B of environment settings, interleaved:
#   scripts/ab_c2_env.sh "GLFSX_QUAD=0" "GLFSX_QUAD=1"
for r in 1 2; do for e in "$@"; do
  for cfg in "--size-gib 1 --block-size 2097152" "--size-gib 0.0625" "--steps 5 --warmup 2"; do
    v=$(env $e python bench.py --no-extras --steps 40 --warmup 5 $cfg | python -c "import json,sys; print(json.loads(sys.stdin.read())['value'])")
    echo "$r $e $cfg $v"
  done
done; done

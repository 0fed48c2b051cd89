#!/bin/bash
# A/B of environment settings on the headline bench, interleaved:
#   scripts/ab_env.sh "GLFSX_FUSED=0" "GLFSX_FUSED=1"
for r in 1 2 3; do for e in "$@"; do
  v=$(env $e python bench.py --no-extras --steps 5 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")
  echo "$r $e $v"
done; done

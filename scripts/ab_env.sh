#!/bin/bash
# Config 2 / 64 MiB / headline A/B of one library under environment settings,
# interleaved: bash scripts/ab_env.sh "GLFSX_QPW=256" "GLFSX_QPW=64" [reps]
A=$1; B=$2; REPS=${3:-3}
for r in $(seq $REPS); do for env in "$A" "$B"; do
  c2=$(env $env timeout -k 10 120 python bench.py --no-extras --size-gib 1 --block-size 2097152 --steps 50 --warmup 5 2>/dev/null | python -c "import json,sys; print(json.loads(sys.stdin.read())['value'])")
  m64=$(env $env timeout -k 10 120 python bench.py --no-extras --size-gib 0.0625 --steps 50 --warmup 5 2>/dev/null | python -c "import json,sys; print(json.loads(sys.stdin.read())['value'])")
  echo "$r [$env] config2 $c2  64MiB $m64"
done; done

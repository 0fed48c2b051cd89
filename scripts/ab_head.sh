#!/bin/bash
# Headline (64 GiB @ 1 MiB) + config 2 (1 GiB @ 2 MiB) A/B of library builds,
# interleaved, each run its own process.  usage: bash scripts/ab_head.sh "a.so b.so" [reps]
LIBS=$1; REPS=${2:-2}
for r in $(seq $REPS); do for lib in $LIBS; do
  h=$(GLFSX_LIB=$lib timeout -k 10 120 python bench.py --no-extras --steps 10 --warmup 2 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'])")
  c=$(GLFSX_LIB=$lib timeout -k 10 120 python bench.py --no-extras --size-gib 1 --block-size 2097152 --steps 50 --warmup 5 2>/dev/null | python -c "import json,sys; print(json.loads(sys.stdin.read())['value'])")
  echo "$r $(basename $lib) head $h config2 $c"
done; done

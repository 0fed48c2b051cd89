#!/bin/bash
# config-2 / 64 MiB A/B of two library builds, interleaved
for r in 1 2; do for lib in "$@"; do
  for cfg in "--size-gib 1 --block-size 2097152" "--size-gib 0.0625"; do
    v=$(GLFSX_LIB=$lib python bench.py --no-extras $cfg --steps 50 --warmup 5 | python -c "import json,sys; print(json.loads(sys.stdin.read())['value'])")
    echo "$r $lib $cfg $v"
  done
done; done

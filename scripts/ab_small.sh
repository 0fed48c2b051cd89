#!/bin/bash
# Config 4 hashing (bench small_blobs leg: 1 M x 4 KiB blobs, device-resident)
# and the headline, A/B of library builds, interleaved.
# usage: bash scripts/ab_small.sh "a.so b.so" [reps]
LIBS=$1; REPS=${2:-2}
for r in $(seq $REPS); do for lib in $LIBS; do
  v=$(GLFSX_LIB=$lib timeout -k 10 200 python bench.py --steps 3 --warmup 1 --cpu-sample-mib 1 --host-rt-gib 0.25 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['small_blobs']['value'], d['config4_end_to_end']['value'])")
  echo "$r $(basename $lib) head/small/config4 $v"
done; done

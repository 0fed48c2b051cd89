#!/bin/bash
# Per-pass cost at different chunks-per-lane G without split mode: the same
# 64 GiB at 256 KiB (G=1), 512 KiB (G=2), 1 MiB (G=4), 2 MiB (G=8) blocks.
for bs in 262144 524288 1048576 2097152; do
  GLFSX_SPLIT_WG=0 timeout -k 10 120 python bench.py --size-gib 64 --block-size $bs --steps 5 --warmup 1 --cpu-sample-mib 1 --host-rt-gib 0 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print($bs, d['value'], r['avg_ms'])"
done

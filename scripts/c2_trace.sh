#!/bin/bash
# rocprofv3 kernel trace of config 2 (1 GiB at 2 MiB blocks) and the
# per-step kernel timeline (scripts/kernel_gaps.py).
export TMPDIR=/tmp
OUT=${1:-gpurun_out/c2}
mkdir -p $OUT
timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $OUT/trace -o run -- python bench.py --no-extras --size-gib 1 --block-size 2097152 --steps 20 --warmup 3 > $OUT/bench.json 2> $OUT/trace.log
python scripts/kernel_gaps.py $OUT/trace > $OUT/gaps.txt

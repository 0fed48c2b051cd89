#!/bin/bash
# round-4 check 19: the config-4 tree blob's Create (115 x 2 MiB) per kernel
# under the default plan and under G1 s3 as two passes, kernel trace
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/tb19
mkdir -p $OUT
timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $OUT/def -o run -- python scripts/r4_plan_sweep.py --shapes 115x2097152 2048 > $OUT/def.json 2> $OUT/def.log || exit $?
GLFSX_DC_MIN=0 GLFSX_FUSED=0 timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $OUT/g1 -o run -- python scripts/r4_plan_sweep.py --shapes 115x2097152 2048 > $OUT/g1.json 2> $OUT/g1.log || exit $?
GLFSX_DC_MIN=0 timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $OUT/dc -o run -- python scripts/r4_plan_sweep.py --shapes 115x2097152 2048 > $OUT/dc.json 2> $OUT/dc.log || exit $?
for d in def g1 dc; do echo "== $d"; cat $OUT/$d.json | tr -d '\n '; echo; python scripts/kernel_gaps.py $OUT/$d 20; done > $OUT/summary.txt

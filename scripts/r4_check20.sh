#!/bin/bash
# round-4 check 20: the config-4 tree blob (115 x 2 MiB) under split targets
# that give G4 s1 (230 wg), G2 s2 (460 wg) and G1 s3 (920 wg) as two passes
# (GLFSX_DC_MIN=0 GLFSX_FUSED=0), per kernel
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/tb20
mkdir -p $OUT
for t in 230 460 920; do
  GLFSX_DC_MIN=0 GLFSX_FUSED=0 timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $OUT/t$t -o run -- python scripts/r4_plan_sweep.py --shapes 115x2097152 $t > $OUT/t$t.json 2> $OUT/t$t.log || exit $?
done
timeout -k 10 200 python scripts/r4_plan_sweep.py --shapes 115x2097152 2048 > $OUT/def.json 2>/dev/null || exit $?
GLFSX_DC_MIN=0 GLFSX_FUSED=0 timeout -k 10 200 python scripts/r4_plan_sweep.py --shapes 115x2097152 230 460 920 > $OUT/all.json 2>/dev/null || exit $?
cat $OUT/def.json $OUT/all.json

#!/bin/bash
# round-4 check 9: few-block Create plans -- the round-4 latency form vs
# non-fused G=1 passes vs the round-3 one-launch post
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
SH=64x2097152,115x2097152,128x1048576,200x2097152
for env in "GLFSX_X=1" "GLFSX_DC_MIN=0 GLFSX_FUSED=0" "GLFSX_DC_MIN=0"; do
  echo "== $env"
  env $env timeout -k 10 200 python -u scripts/r4_plan_sweep.py --shapes $SH 2048 2>/dev/null \
    | python -c "import json,sys; d=json.load(sys.stdin); print({k: v['2048']['GiBps'] for k, v in d.items()})" || exit 1
done

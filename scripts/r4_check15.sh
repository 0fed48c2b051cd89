#!/bin/bash
# round-4 check 15: config 2 (512 x 2 MiB) under k_pass_dc's fine-item share
# (GLFSX_DC_FINE) and the split target, interleaved processes
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/r4_c2fine.log
for r in 1 2; do
for env in "GLFSX_DC_FINE=4" "GLFSX_DC_FINE=0" "GLFSX_DC_FINE=2" "GLFSX_DC_FINE=8"; do
  echo "$env $(env $env timeout -k 10 120 python -u scripts/r4_plan_sweep.py --shapes 512x2097152 2048 3072 2>/dev/null | python -c 'import json,sys; d=json.load(sys.stdin); print({t: v["GiBps"] for t, v in d["512x2048K"].items()})')" | tee -a gpurun_out/r4_c2fine.log
done
done

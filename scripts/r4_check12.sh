#!/bin/bash
# round-4 check 12: host feeds, NUMA placement A/B -- library copy pool on the
# GPU's node (GLFSX_NUMA) and the whole process there (FEED_NUMA)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/r4_numa2.jsonl
for r in 1 2; do
for env in "GLFSX_NUMA=0 FEED_NUMA=0" "GLFSX_NUMA=1 FEED_NUMA=0" "GLFSX_NUMA=1 FEED_NUMA=1"; do
  env $env timeout -k 10 150 python -u scripts/r4_feed_sweep.py >> gpurun_out/r4_numa2.jsonl 2>/dev/null || exit 1
  tail -1 gpurun_out/r4_numa2.jsonl
done
done

#!/bin/bash
# round-4 check 10: file-feed sensitivity to reader threads, slots and batch size
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/r4_feed.jsonl
for env in "GLFSX_X=1" "GLFSX_READ_THREADS=4" "GLFSX_READ_THREADS=8" "GLFSX_SLOTS=4" \
           "GLFSX_BATCH_MIB=32" "GLFSX_BATCH_MIB=128" "GLFSX_X=1"; do
  env $env timeout -k 10 150 python -u scripts/r4_feed_sweep.py >> gpurun_out/r4_feed.jsonl 2>/dev/null || exit 1
  tail -1 gpurun_out/r4_feed.jsonl
done

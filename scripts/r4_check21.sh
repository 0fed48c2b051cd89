#!/bin/bash
# round-4 check 21: config 4 one call, the DEK pass queued before the layout
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 400 --timeout-method thread \
  tests/test_gpu_tree_read.py tests/test_gpu_small_bs.py tests/test_gpu_node.py \
  > gpurun_out/r4_t21.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r4_t21.log; exit 1; }
tail -1 gpurun_out/r4_t21.log
timeout -k 10 700 python -u scripts/ab_small.py 3 "GLFSX_DEK_FIRST=1" \
  "GLFSX_DEK_FIRST=0" \
  > gpurun_out/r4_ab21.log 2>&1 || { echo "ab failed"; tail -20 gpurun_out/r4_ab21.log; exit 1; }
tail -4 gpurun_out/r4_ab21.log
bash scripts/r4_c4tl.sh

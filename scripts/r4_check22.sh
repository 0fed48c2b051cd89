#!/bin/bash
# round-4 check 22: config 4 one call, the CID pass in two groups with the tree blocks beside the second
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 400 --timeout-method thread \
  tests/test_gpu_tree_read.py tests/test_gpu_small_bs.py tests/test_gpu_node.py \
  > gpurun_out/r4_t22.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r4_t22.log; exit 1; }
tail -1 gpurun_out/r4_t22.log
timeout -k 10 700 python -u scripts/ab_small.py 3 "GLFSX_TREE_SPLIT=85" \
  "GLFSX_TREE_SPLIT=0" "GLFSX_TREE_SPLIT=70" \
  > gpurun_out/r4_ab22.log 2>&1 || { echo "ab failed"; tail -20 gpurun_out/r4_ab22.log; exit 1; }
tail -4 gpurun_out/r4_ab22.log
bash scripts/r4_c4tl.sh

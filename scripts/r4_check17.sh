#!/bin/bash
# round-4 check 17: config 4's one call with the layout and static lines
# beside the DEK pass (the total in pinned memory, no copy kernel) -- the
# tree tests, then A/B raised priority on / off / the first round-4 order,
# then a timeline
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 400 --timeout-method thread \
  tests/test_gpu_tree_read.py tests/test_gpu_small_bs.py tests/test_gpu_node.py \
  > gpurun_out/r4_t17.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r4_t17.log; exit 1; }
tail -1 gpurun_out/r4_t17.log
timeout -k 10 700 python -u scripts/ab_small.py 3 "GLFSX_TREE_PRIO=1" \
  "GLFSX_TREE_PRIO=0" "GLFSX_TREE_BESIDE=0 GLFSX_TREE_ON_A=0" \
  > gpurun_out/r4_ab17.log 2>&1 || { echo "ab failed"; tail -20 gpurun_out/r4_ab17.log; exit 1; }
tail -4 gpurun_out/r4_ab17.log
bash scripts/r4_c4tl.sh

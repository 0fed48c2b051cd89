#!/bin/bash
# round-4 check 7: full gpu suite, then config-4 A/B (previous library vs this one)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q -m gpu --timeout 400 --timeout-method thread tests \
  > gpurun_out/r4_t7.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r4_t7.log; exit 1; }
tail -2 gpurun_out/r4_t7.log
timeout -k 10 700 python -u scripts/ab_small.py 3 "GLFSX_LIB=glfs_amd/libglfsx_head.so" "GLFSX_X=1" "GLFSX_TREE_HEX=0" > gpurun_out/r4_ab7.log 2>&1
rc=$?; tail -4 gpurun_out/r4_ab7.log; exit $rc

#!/bin/bash
# round-4 check 5: tests touched by the plan / tree-line changes, then A/B of
# the HEAD library vs the new one (and the two-phase tree-line variant)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_tree_read.py tests/test_gpu_small_bs.py tests/test_gpu_parity.py tests/test_gpu_writer.py \
  > gpurun_out/r4_t5.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r4_t5.log; exit 1; }
tail -2 gpurun_out/r4_t5.log
SH=64x2097152,115x2097152,128x1048576,200x2097152,512x2097152,1024x1048576
for lib in glfs_amd/libglfsx_head.so glfs_amd/libglfsx.so; do
  GLFSX_LIB=$lib timeout -k 10 200 python -u scripts/r4_plan_sweep.py --shapes $SH 2048 > gpurun_out/r4_sw5_$(basename $lib .so).json 2>/dev/null || exit 1
done
timeout -k 10 700 python -u scripts/ab_small.py 3 "GLFSX_LIB=glfs_amd/libglfsx_head.so" "GLFSX_X=1" "GLFSX_LIB=glfs_amd/libglfsx_ph2.so" > gpurun_out/r4_ab5.log 2>&1
rc=$?; tail -4 gpurun_out/r4_ab5.log; exit $rc

#!/bin/bash
# round-4 check 8: tree tests, config-4 A/B of the half-workgroup static
# line writer, and the one-process N=4 bench rehearsal with its extras
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_tree_read.py tests/test_gpu_small_bs.py > gpurun_out/r4_t8.log 2>&1 \
  || { echo "tests failed"; tail -40 gpurun_out/r4_t8.log; exit 1; }
tail -1 gpurun_out/r4_t8.log
timeout -k 10 500 python -u scripts/ab_small.py 3 "GLFSX_TREE_HALF=1" "GLFSX_TREE_HALF=0" > gpurun_out/r4_ab8.log 2>&1 \
  || { echo "ab failed"; tail -20 gpurun_out/r4_ab8.log; exit 1; }
tail -2 gpurun_out/r4_ab8.log
timeout -k 10 400 python -u bench.py --gpus 4 --rehearse --size-gib 16 --steps 2 --warmup 1 \
  > gpurun_out/r4_n4.json 2> gpurun_out/r4_n4.err
rc=$?; echo "n4 rc=$rc"; tail -c 2500 gpurun_out/r4_n4.json; exit $rc

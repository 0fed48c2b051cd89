#!/bin/bash
# round-4 check 3: config-4 A/B (pre-hex-fusion library vs HEAD, GLFSX_TREE_HEX=0/1)
# and the split-plan sweep for the tree-blob shape
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/r4_plan_sweep.py 2048 128 100 64 32 > gpurun_out/r4_sweep2.json 2> gpurun_out/r4_sweep2.err
rc=$?; echo "sweep rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 800 python -u scripts/ab_small.py 3 "GLFSX_LIB=glfs_amd/libglfsx_pre.so" "GLFSX_TREE_HEX=1" "GLFSX_TREE_HEX=0" > gpurun_out/r4_ab_hex.log 2>&1
rc=$?; echo "ab rc=$rc"; tail -5 gpurun_out/r4_ab_hex.log; exit $rc

#!/bin/bash
# round-4 check 4: split-plan sweep over Create shapes (blocks x block size)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u scripts/r4_plan_sweep.py --shapes 32x2097152,64x2097152,115x2097152,200x2097152,256x2097152,384x2097152,512x2097152,64x1048576,128x1048576,256x1048576,512x1048576,1024x1048576 2048 1024 512 256 128 64 > gpurun_out/r4_sweep3.json 2> gpurun_out/r4_sweep3.err
rc=$?; echo "sweep rc=$rc"; tail -3 gpurun_out/r4_sweep3.err; exit $rc

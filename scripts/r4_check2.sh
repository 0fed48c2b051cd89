#!/bin/bash
# round-4 check 2: the full gpu suite, then a default bench line
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v -m gpu --timeout 400 --timeout-method thread tests \
  > gpurun_out/r4_t2.log 2>&1 || { echo "tests failed rc=$?"; tail -60 gpurun_out/r4_t2.log; exit 1; }
tail -3 gpurun_out/r4_t2.log
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 > gpurun_out/r4_b2.json 2> gpurun_out/r4_b2.err
rc=$?; echo "bench rc=$rc"; tail -c 1500 gpurun_out/r4_b2.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/r4_plan_sweep.py > gpurun_out/r4_sweep.json 2> gpurun_out/r4_sweep.err
rc=$?; echo "sweep rc=$rc"; cat gpurun_out/r4_sweep.json; exit $rc

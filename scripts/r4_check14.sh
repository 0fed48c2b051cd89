#!/bin/bash
# round-4 check 14: full gpu suite, default bench line, config-4 A/B of the
# host's poll bound (GLFSX_SPIN_US)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q -m gpu --timeout 400 --timeout-method thread tests \
  > gpurun_out/r4_t14.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r4_t14.log; exit 1; }
tail -1 gpurun_out/r4_t14.log
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 > gpurun_out/r4_b14.json 2> gpurun_out/r4_b14.err \
  || { echo "bench failed"; tail -20 gpurun_out/r4_b14.err; exit 1; }
echo "bench ok"
timeout -k 10 500 python -u scripts/ab_small.py 3 "GLFSX_SPIN_US=2000" "GLFSX_SPIN_US=20000" > gpurun_out/r4_ab14.log 2>&1
rc=$?; tail -3 gpurun_out/r4_ab14.log; exit $rc

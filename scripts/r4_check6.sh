#!/bin/bash
# round-4 check 6: full gpu suite, then the rocprofv3 passes behind profiles/r4/
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q -m gpu --timeout 400 --timeout-method thread tests \
  > gpurun_out/r4_t6.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r4_t6.log; exit 1; }
tail -2 gpurun_out/r4_t6.log
bash scripts/profile_r4.sh gpurun_out/prof_r4
rc=$?; echo "profile rc=$rc"; ls gpurun_out/prof_r4; exit $rc

#!/bin/bash
# The round-end check on a GPU box: the whole -m gpu suite, smoke(), and the
# default bench line (gpurun_out/r4_t18.log, r4_s18.log, r4_b18.json)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q -m gpu --timeout 400 --timeout-method thread tests \
  > gpurun_out/r4_t18.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r4_t18.log; exit 1; }
tail -1 gpurun_out/r4_t18.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" \
  > gpurun_out/r4_s18.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/r4_s18.log; exit 1; }
tail -1 gpurun_out/r4_s18.log
timeout -k 10 400 python -u bench.py > gpurun_out/r4_b18.json 2> gpurun_out/r4_b18.err \
  || { echo "bench failed"; tail -20 gpurun_out/r4_b18.err; exit 1; }
echo "bench ok"

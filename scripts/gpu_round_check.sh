#!/bin/bash
# The round-end check on a GPU box: the whole -m gpu suite (the files named
# in $2 first), smoke(), and the default bench line.  $1 = a tag for the
# output names (gpurun_out/<tag>_t.log, _s.log, _b.json).
tag=${1:-check}
first=${2:-}
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest -x -v -m gpu --timeout 400 --timeout-method thread $first tests \
  > gpurun_out/${tag}_t.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/${tag}_t.log; exit 1; }
tail -1 gpurun_out/${tag}_t.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" \
  > gpurun_out/${tag}_s.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/${tag}_s.log; exit 1; }
tail -1 gpurun_out/${tag}_s.log
timeout -k 10 400 python -u bench.py > gpurun_out/${tag}_b.json 2> gpurun_out/${tag}_b.err \
  || { echo "bench failed"; tail -20 gpurun_out/${tag}_b.err; exit 1; }
echo "bench ok"

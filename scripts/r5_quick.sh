#!/bin/bash
# Round-5 quick GPU check: the tree / one-shot / knob tests, then the legs
# that changed (config 4 routes, PostBlob latency and concurrency, config 2).
# $1 = output tag.
tag=${1:-q}
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread \
  tests/test_gpu_tree_read.py tests/test_gpu_one.py tests/test_gpu_knobs.py \
  > gpurun_out/${tag}_t.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/${tag}_t.log; exit 1; }
tail -1 gpurun_out/${tag}_t.log
for leg in config4all postblob postblob config2; do
  timeout -k 10 300 python -u scripts/legs.py $leg >> gpurun_out/${tag}_${leg}.json \
    2> gpurun_out/${tag}_${leg}.err || { echo "leg $leg failed"; tail -20 gpurun_out/${tag}_${leg}.err; exit 1; }
done
echo "legs ok"

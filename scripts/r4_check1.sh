#!/bin/bash
# round-4 first GPU check: new/changed tests, then a default bench line
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest -x -v --timeout 400 --timeout-method thread \
  tests/test_gpu_small_bs.py tests/test_gpu_read_fd.py tests/test_gpu_devices.py \
  tests/test_gpu_fused.py tests/test_gpu_multi.py tests/test_gpu_shard_mp.py \
  > gpurun_out/r4_t1.log 2>&1 || { echo "tests failed rc=$?"; tail -40 gpurun_out/r4_t1.log; exit 1; }
tail -5 gpurun_out/r4_t1.log
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 > gpurun_out/r4_b1.json 2> gpurun_out/r4_b1.err
rc=$?; echo "bench rc=$rc"; tail -c 3000 gpurun_out/r4_b1.json; exit $rc

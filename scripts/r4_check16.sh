#!/bin/bash
# round-4 check 16: k_node (a latency-form post in one launch) -- its tests
# and the parity / fused / one-shot suites, then Create A/B GLFSX_NODE=1 vs 0
# (config 2, the config-4 tree blob, one 2 MiB block; HIP events), then
# config 4 A/B
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_node.py tests/test_gpu_parity.py tests/test_gpu_fused.py tests/test_gpu_one.py \
  > gpurun_out/r4_t16.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r4_t16.log; exit 1; }
tail -1 gpurun_out/r4_t16.log
: > gpurun_out/r4_node_ab.log
for r in 1 2 3; do
for env in "GLFSX_NODE=1" "GLFSX_NODE=0"; do
  echo "$env $(env $env timeout -k 10 120 python -u scripts/r4_plan_sweep.py --shapes 512x2097152,115x2097152,1x2097152,16x1048576 2048 2>/dev/null | python -c 'import json,sys; d=json.load(sys.stdin); print({k: v["2048"]["ms"] for k, v in d.items()})')" | tee -a gpurun_out/r4_node_ab.log
done
done
timeout -k 10 500 python -u scripts/ab_small.py 2 "GLFSX_NODE=1" "GLFSX_NODE=0" > gpurun_out/r4_ab16.log 2>&1
rc=$?; tail -3 gpurun_out/r4_ab16.log; exit $rc

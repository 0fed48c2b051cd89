#!/bin/bash
# Run named GPU steps on the gpurun box, each under its own time limit.
# Usage: scripts/gpu_steps.sh "name:seconds:command" ...
# A step that ends with a test failure (rc 1) lets later steps run; any other
# nonzero status (timeout 124/137, abort 134, segfault 139, ...) stops the
# script so nothing more touches a possibly faulted GPU.
mkdir -p gpurun_out
for spec in "$@"; do
  name="${spec%%:*}"; rest="${spec#*:}"; secs="${rest%%:*}"; cmd="${rest#*:}"
  echo "[$(date +%T)] start $name ($secs s): $cmd" >> gpurun_out/steps.log
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "[$(date +%T)] end $name rc=$rc" >> gpurun_out/steps.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    echo "stopping after $name rc=$rc" >> gpurun_out/steps.log
    exit $rc
  fi
done
exit 0

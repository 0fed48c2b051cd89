#!/bin/bash
# Submit one gpurun call; when no box/slot is free (exit 3: nothing ran,
# nothing charged) wait and submit the same call again.  Any other status,
# including a failed or timed-out command, is returned as is.
# usage: scripts/gpurun_wait.sh TIMEOUT 'command'
T=$1; shift
for i in $(seq 30); do
  /usr/local/graft/bin/gpurun --timeout "$T" -- "$@"
  rc=$?
  [ $rc -ne 3 ] && exit $rc
  sleep 60
done
exit 3

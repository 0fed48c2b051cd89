#!/bin/bash
# round-4: config 4 one-call timeline (both streams) under rocprofv3
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/c4tl
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -f csv -d $OUT/tr -o run -- python scripts/legs.py config4one > $OUT/c4one.json 2> $OUT/c4one.log || exit $?
python scripts/c4_timeline.py $OUT/tr > $OUT/timeline.txt

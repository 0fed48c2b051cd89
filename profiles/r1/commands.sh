#!/bin/bash
# rocprofv3 passes for round-1 profiles (run on the GPU box from the repo root).
# Each pass is its own process; PMC passes use --kernel-trace only.
set -e
export TMPDIR=/tmp
OUT=gpurun_out/prof
mkdir -p $OUT
B="python bench.py --no-extras --steps 3 --warmup 1"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/trace -o run -- $B > $OUT/trace.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -f csv -d $OUT/fetch -o run -- $B --size-gib 16 > $OUT/fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -f csv -d $OUT/write -o run -- $B --size-gib 16 > $OUT/write.log 2>&1
timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM --kernel-trace -f csv -d $OUT/sq -o run -- $B --size-gib 16 > $OUT/sq.log 2>&1
timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_BUSY_CYCLES --kernel-trace -f csv -d $OUT/kb -o run -- tools/kbench 8 > $OUT/kb.log 2>&1

#!/bin/bash
# rocprofv3 passes over the secondary legs (scripts/legs.py): kernel trace +
# stats, then one SQ counter pass (VALU instructions, busy cycles, clocks).
set -e
export TMPDIR=/tmp
OUT=${1:-gpurun_out/prof_legs}
mkdir -p $OUT
timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $OUT/trace -o run -- python scripts/legs.py > $OUT/legs.json 2> $OUT/trace.log
timeout -s KILL 200 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM SQ_INSTS_LDS SQ_BUSY_CYCLES --kernel-trace -f csv -d $OUT/sq -o run -- python scripts/legs.py > $OUT/sq.log 2>&1
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --kernel-trace -f csv -d $OUT/fetch -o run -- python scripts/legs.py > $OUT/fetch.log 2>&1
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --kernel-trace -f csv -d $OUT/write -o run -- python scripts/legs.py > $OUT/write.log 2>&1
python scripts/prof_summary.py $OUT $OUT/summary.json > $OUT/summary.txt

#!/bin/bash
# One SQ counter pass (VALU instructions, busy cycles, clocks) over the
# headline kernels and the secondary legs; summary in $OUT/summary.txt.
set -e
export TMPDIR=/tmp
OUT=${1:-gpurun_out/sq_quick}
mkdir -p $OUT
timeout -s KILL 200 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES --kernel-trace -f csv -d $OUT/sq -o run -- python bench.py --no-extras --steps 2 --warmup 1 > $OUT/sq.log 2>&1
timeout -s KILL 200 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES --kernel-trace -f csv -d $OUT/sql -o run -- python scripts/legs.py > $OUT/sql.log 2>&1
python scripts/prof_summary.py $OUT $OUT/summary.json > $OUT/summary.txt

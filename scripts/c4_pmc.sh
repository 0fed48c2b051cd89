#!/bin/bash
# Round 6: counters over config 4's one-call route (scripts/legs.py
# config4one), to see where the tree blob's latency-form passes
# (k_pass<4, false, true, 0>, 230 workgroups) spend their time against the
# bulk passes: SQ issue/wait counters in one pass, LDS bank conflicts in a
# second.
export TMPDIR=/tmp
OUT=${1:-gpurun_out/c4_pmc}
mkdir -p $OUT
SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE"
timeout -s KILL 200 rocprofv3 --pmc $SQ --kernel-trace -f csv -d $OUT/sq -o run -- python scripts/legs.py config4one > $OUT/sq.log 2>&1 || exit $?
timeout -s KILL 200 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU --kernel-trace -f csv -d $OUT/lds -o run -- python scripts/legs.py config4one > $OUT/lds.log 2>&1 || exit $?
python scripts/prof_summary.py $OUT $OUT/summary.json > $OUT/summary.txt
echo "c4 pmc ok"

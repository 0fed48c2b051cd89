#!/bin/bash
# rocprofv3 passes behind profiles/r6/final/ (run on the GPU box from the repo root):
#   trace  : the default bench command itself, --kernel-trace --stats (its
#            HIP-event roofline.avg_ms, its in-run clock and rocprof's
#            per-kernel mean come from the same process and launches)
#   fetch / write / sq : PMC passes, one counter group each, --kernel-trace
#            only, over the headline launches (--no-extras)
#   c2     : config 2 (1 GiB at 2 MiB) kernel trace, per-step timeline
#   c4     : config 4 one-call route kernel trace, per-call timeline
export TMPDIR=/tmp
OUT=${1:-gpurun_out/prof_r6final}
mkdir -p $OUT
B="python bench.py --no-extras --steps 3 --warmup 1"
timeout -k 10 500 rocprofv3 --kernel-trace --stats -f csv -d $OUT/trace -o run -- python bench.py > $OUT/bench.json 2> $OUT/trace.log || exit $?
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --kernel-trace -f csv -d $OUT/fetch -o run -- $B > $OUT/fetch.log 2>&1 || exit $?
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --kernel-trace -f csv -d $OUT/write -o run -- $B > $OUT/write.log 2>&1 || exit $?
timeout -s KILL 200 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM SQ_INSTS_LDS SQ_BUSY_CYCLES --kernel-trace -f csv -d $OUT/sq -o run -- $B > $OUT/sq.log 2>&1 || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $OUT/c2 -o run -- python bench.py --no-extras --size-gib 1 --block-size 2097152 --steps 20 --warmup 3 > $OUT/c2_bench.json 2> $OUT/c2.log || exit $?
python scripts/kernel_gaps.py $OUT/c2 3 k_pass_dc > $OUT/c2_gaps.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/c4 -o run -- python scripts/legs.py config4one > $OUT/c4.json 2> $OUT/c4.log || exit $?
python scripts/kernel_gaps.py $OUT/c4 3 "k_small_q<4, false" > $OUT/c4_gaps.txt
python scripts/prof_summary.py $OUT $OUT/summary.json > $OUT/summary.txt
python scripts/pmc_traffic.py $OUT/summary.json $OUT/pmc_traffic.json > /dev/null
echo "profile ok"

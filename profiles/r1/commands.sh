#!/bin/bash
# rocprofv3 passes behind profiles/<round>/ (run on the GPU box from the repo
# root): usage  bash scripts/profile.sh [OUT=gpurun_out/prof]
#  trace : the default bench command itself under --kernel-trace --stats, so
#          bench's HIP-event roofline.avg_ms and rocprof's per-kernel average
#          come from the same process and launches
#  fetch / write / sq : PMC passes (one counter group each, --kernel-trace
#          only, never combined with other trace domains) over the same
#          64 GiB launches without the extra legs
#  kb    : tools/kbench (VALU ceiling of the DEK code shape)
set -e
export TMPDIR=/tmp
OUT=${1:-gpurun_out/prof}
mkdir -p $OUT
B="python bench.py --no-extras --steps 3 --warmup 1"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $OUT/trace -o run -- python bench.py > $OUT/bench.json 2> $OUT/trace.log
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --kernel-trace -f csv -d $OUT/fetch -o run -- $B > $OUT/fetch.log 2>&1
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --kernel-trace -f csv -d $OUT/write -o run -- $B > $OUT/write.log 2>&1
timeout -s KILL 200 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM SQ_INSTS_LDS SQ_BUSY_CYCLES --kernel-trace -f csv -d $OUT/sq -o run -- $B > $OUT/sq.log 2>&1
if [ -x tools/kbench ]; then
  timeout -s KILL 200 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_BUSY_CYCLES --kernel-trace -f csv -d $OUT/kb -o run -- tools/kbench 8 > $OUT/kb.log 2>&1
fi
python scripts/prof_summary.py $OUT $OUT/summary.json > $OUT/summary.txt
# secondary legs (config 4 small blobs, read side) alone: legs/
#   bash scripts/profile_legs.sh gpurun_out/prof_legs
# per-launch HBM traffic for bench.py's roofline.traffic:
#   python scripts/pmc_traffic.py profiles/r1/summary.json profiles/pmc_traffic.json

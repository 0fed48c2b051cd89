#!/bin/bash
# A/B of the one-shot descriptor staged in LDS (libglfsx.so) against fields
# read where used (libglfsx_desc0.so, -DGLFSX_DESC_LDS=0): PostBlob latency
# and concurrency, interleaved, 3 reps.
export TMPDIR=/tmp
OUT=${1:-gpurun_out/ab_desc}
mkdir -p $OUT
for rep in 1 2 3; do
  for v in desc0 cur; do
    L=glfs_amd/libglfsx_$v.so
    [ $v = cur ] && L=glfs_amd/libglfsx.so
    GLFSX_LIB=$L timeout -k 10 120 python scripts/legs.py postblob > $OUT/pb_${v}_$rep.json 2>> $OUT/err.log || exit $?
  done
done
echo "ab ok"

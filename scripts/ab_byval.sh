#!/bin/bash
# A/B of the one-shot descriptor passed by value for a one-post launch (libglfsx.so) against
# the pinned descriptor array (libglfsx_bv0.so, -DGLFSX_ONE_BYVAL=0): PostBlob latency
# and concurrency, interleaved, 3 reps; head = the previous commit (neither the
# by-value launch nor the zero-initialised k_med_cid staging).
export TMPDIR=/tmp
OUT=${1:-gpurun_out/ab_byval}
mkdir -p $OUT
for rep in 1 2 3; do
  for v in head bv0 cur; do
    L=glfs_amd/libglfsx_$v.so
    [ $v = cur ] && L=glfs_amd/libglfsx.so
    GLFSX_LIB=$L timeout -k 10 120 python scripts/legs.py postblob > $OUT/pb_${v}_$rep.json 2>> $OUT/err.log || exit $?
  done
done
echo "ab ok"

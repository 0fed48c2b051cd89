#!/bin/bash
# A/B of the one-shot chunk loop unrolled 16x (libglfsx.so) against 1x / 2x / 4x
# (libglfsx_u1/u2/u4.so, -DGLFSX_ONE_UNROLL=N; the instruction cache): PostBlob latency
export TMPDIR=/tmp
OUT=${1:-gpurun_out/ab_unroll}
mkdir -p $OUT
for rep in 1 2 3; do
  for v in cur u1 u2 u4; do
    L=glfs_amd/libglfsx_$v.so
    [ $v = cur ] && L=glfs_amd/libglfsx.so
    GLFSX_LIB=$L timeout -k 10 120 python scripts/legs.py postblob > $OUT/pb_${v}_$rep.json 2>> $OUT/err.log || exit $?
  done
done
echo "ab ok"

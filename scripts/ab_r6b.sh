#!/bin/bash
# A/B of the prefetching quad chains (libglfsx.so) against the previous
# commit's build (libglfsx_r6base.so), interleaved: PostBlob latency,
# config 2, and the index-node chain (quad_lat.py under a kernel trace).
export TMPDIR=/tmp
OUT=${1:-gpurun_out/ab_r6b}
mkdir -p $OUT
for rep in 1 2 3; do
  for v in r6base cur; do
    L=glfs_amd/libglfsx_$v.so
    [ $v = cur ] && L=glfs_amd/libglfsx.so
    GLFSX_LIB=$L timeout -k 10 120 python scripts/legs.py postblob > $OUT/pb_${v}_$rep.json 2>> $OUT/err.log || exit $?
    GLFSX_LIB=$L timeout -k 10 120 python scripts/legs.py config2 > $OUT/c2_${v}_$rep.json 2>> $OUT/err.log || exit $?
  done
done
for v in r6base cur; do
  L=glfs_amd/libglfsx_$v.so
  [ $v = cur ] && L=glfs_amd/libglfsx.so
  GLFSX_LIB=$L timeout -k 10 120 rocprofv3 --kernel-trace --stats -f csv -d $OUT/ql_$v -o run -- python scripts/quad_lat.py > $OUT/ql_$v.log 2>&1 || exit $?
  python scripts/quad_lat_sum.py $OUT/ql_$v > $OUT/quad_lat_$v.json || exit $?
done
echo "ab ok"

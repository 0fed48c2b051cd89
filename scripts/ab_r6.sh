#!/bin/bash
# Round-6 A/B on one box (run from the repo root on the GPU box), libraries
# interleaved: base = the previous commit's build (libglfsx_r6base.so),
# qasm0 = this build without the asm quad rounds (-DGLFSX_QASM=0), cur = this
# build.  Per library: the index-node chain (quad_lat.py under a kernel
# trace), PostBlob latency, config 2 and Concat (scripts/legs.py).
export TMPDIR=/tmp
OUT=${1:-gpurun_out/ab_r6}
mkdir -p $OUT
for rep in 1 2; do
  for v in r6base qasm0 cur; do
    L=glfs_amd/libglfsx_$v.so
    [ $v = cur ] && L=glfs_amd/libglfsx.so
    GLFSX_LIB=$L timeout -k 10 120 python scripts/legs.py postblob > $OUT/pb_${v}_$rep.json 2>> $OUT/err.log || exit $?
    GLFSX_LIB=$L timeout -k 10 120 python scripts/legs.py config2 > $OUT/c2_${v}_$rep.json 2>> $OUT/err.log || exit $?
    GLFSX_LIB=$L timeout -k 10 120 python scripts/legs.py concat > $OUT/cc_${v}_$rep.json 2>> $OUT/err.log || exit $?
    echo "rep $rep $v done"
  done
done
for v in r6base qasm0 cur; do
  L=glfs_amd/libglfsx_$v.so
  [ $v = cur ] && L=glfs_amd/libglfsx.so
  GLFSX_LIB=$L timeout -k 10 120 rocprofv3 --kernel-trace --stats -f csv -d $OUT/ql_$v -o run -- python scripts/quad_lat.py > $OUT/ql_$v.log 2>&1 || exit $?
done
echo "ab ok"

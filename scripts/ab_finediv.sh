#!/bin/bash
# A/B of config 2 over k_pass_dc's fine-item share (GLFSX_DC_FINE_DIV: the
# last ceil(m / div) messages of each work list as fine CID items; default
# 4 = libglfsx.so; variants fd1 / fd2 / fd8), interleaved -- round 6.
export TMPDIR=/tmp
OUT=${1:-gpurun_out/ab_finediv}
mkdir -p $OUT
for rep in 1 2 3; do
  for v in cur fd1 fd2 fd8; do
    L=glfs_amd/libglfsx_$v.so
    [ $v = cur ] && L=glfs_amd/libglfsx.so
    GLFSX_LIB=$L timeout -k 10 120 python scripts/legs.py config2 > $OUT/c2_${v}_$rep.json 2>> $OUT/err.log || exit $?
  done
done
echo "ab ok"

#!/bin/bash
# A/B of the quad-layout round with every row rotation folded into its first
# consumer (libglfsx_qf.so, -DGLFSX_QFOLD=1) against QROUND_ASM (libglfsx.so):
# PostBlob latency / concurrency and config 2 (its index-node chain),
# interleaved, 3 reps -- round 6.
export TMPDIR=/tmp
OUT=${1:-gpurun_out/ab_qfold}
mkdir -p $OUT
for rep in 1 2 3; do
  for v in cur qf; do
    L=glfs_amd/libglfsx_$v.so
    [ $v = cur ] && L=glfs_amd/libglfsx.so
    GLFSX_LIB=$L timeout -k 10 120 python scripts/legs.py postblob > $OUT/pb_${v}_$rep.json 2>> $OUT/err.log || exit $?
    GLFSX_LIB=$L timeout -k 10 120 python scripts/legs.py config2 > $OUT/c2_${v}_$rep.json 2>> $OUT/err.log || exit $?
  done
done
for v in cur qf; do
  L=glfs_amd/libglfsx_$v.so
  [ $v = cur ] && L=glfs_amd/libglfsx.so
  GLFSX_LIB=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $OUT/tr_$v -o run -- python bench.py --no-extras --size-gib 1 --block-size 2097152 --steps 20 --warmup 3 > $OUT/tr_$v.json 2> $OUT/tr_$v.log || exit $?
  python scripts/kernel_gaps.py $OUT/tr_$v 3 k_pass_dc > $OUT/gaps_$v.txt || exit $?
done
echo "ab ok"

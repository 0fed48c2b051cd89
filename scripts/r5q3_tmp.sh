export TMPDIR=/tmp
bash scripts/gpu_round_check.sh r5d || exit 1
for r in 1 2; do
  GLFSX_LIB=$PWD/glfs_amd/libglfsx_base.so timeout -k 10 200 python scripts/legs.py postblob > gpurun_out/r5d_pb_base_$r.json || exit 1
  timeout -k 10 200 python scripts/legs.py postblob > gpurun_out/r5d_pb_new_$r.json || exit 1
done
echo legs ok

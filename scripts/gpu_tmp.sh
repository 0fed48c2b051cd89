export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests/test_gpu_one.py > gpurun_out/q6_t.log 2>&1 || { tail -20 gpurun_out/q6_t.log; exit 1; }
tail -1 gpurun_out/q6_t.log
for r in 1 2; do
  GLFSX_LIB=$PWD/glfs_amd/libglfsx_base.so timeout -k 10 200 python scripts/legs.py postblob > gpurun_out/q6_base_$r.json || exit 1
  timeout -k 10 200 python scripts/legs.py postblob > gpurun_out/q6_new_$r.json || exit 1
done
echo ok

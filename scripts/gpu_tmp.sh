export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests/test_gpu_one.py tests/test_gpu_node.py > gpurun_out/q7_t.log 2>&1 || { tail -20 gpurun_out/q7_t.log; exit 1; }
tail -1 gpurun_out/q7_t.log
for r in 1 2; do
 for v in pf new; do
  if [ $v = pf ]; then export GLFSX_LIB=$PWD/glfs_amd/libglfsx_pf.so; else unset GLFSX_LIB; fi
  for sz in 4096 65536 1048576 2097152; do timeout -k 10 120 python scripts/one_trace.py $sz > gpurun_out/q7_${v}_${r}_$sz.json || exit 1; done
  timeout -k 10 200 python scripts/legs.py config2 > gpurun_out/q7_${v}_${r}_c2.json || exit 1
 done
done
unset GLFSX_LIB
timeout -k 10 200 rocprofv3 --kernel-trace -f csv -d gpurun_out/q7_c2new -o run -- python bench.py --no-extras --size-gib 1 --block-size 2097152 --steps 20 --warmup 3 > gpurun_out/q7_c2new.json 2> gpurun_out/q7_c2new.log || exit 1
python scripts/kernel_gaps.py gpurun_out/q7_c2new 3 k_pass_dc > gpurun_out/q7_c2new_gaps.txt
echo ok

export TMPDIR=/tmp
mkdir -p gpurun_out/one_r6
for sz in 0 4096 65536; do
  GLFSX_LIB=glfs_amd/libglfsx_onet.so timeout -k 10 120 python scripts/one_trace.py $sz > gpurun_out/one_r6/phase_$sz.json 2>>gpurun_out/one_r6/err.log || exit $?
  timeout -k 10 120 rocprofv3 --kernel-trace -f csv -d gpurun_out/one_r6/tr_$sz -o run -- python scripts/one_trace.py $sz > gpurun_out/one_r6/run_$sz.json 2>>gpurun_out/one_r6/err.log || exit $?
  python scripts/one_trace.py --report gpurun_out/one_r6/tr_$sz $sz > gpurun_out/one_r6/report_$sz.json || exit $?
done
echo one ok

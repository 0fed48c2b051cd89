export TMPDIR=/tmp
bash scripts/gpu_round_check.sh r5e tests/test_gpu_one.py || exit 1
echo ok

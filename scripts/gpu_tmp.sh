export TMPDIR=/tmp
bash scripts/gpu_round_check.sh r5f || exit 1
echo ok

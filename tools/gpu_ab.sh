# Development GPU pass: index/dist parity tests, then shard-size sweeps under A/B settings.
# Each GPU step has its own time limit and the first failure ends the script.
# Usage: bash tools/gpu_ab.sh [tests|notests] "ENV=.. ENV2=.." "ENV=.." ...
set -u
mkdir -p gpurun_out
if [ "${1:-tests}" = tests ]; then
  timeout -k 10 400 python -u -m pytest tests/test_gpu_index.py tests/test_gpu_dist.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_idx.log 2>&1
  rc=$?; tail -3 gpurun_out/t_idx.log; [ $rc -ne 0 ] && exit $rc
fi
shift || true
i=0
for envs in "$@"; do
  i=$((i+1))
  echo "=== [$i] ${envs:-defaults}"
  env $envs timeout -k 10 150 python -u tools/sweep.py ${ROWS:-1250000 2500000 5000000 10000000} > gpurun_out/sweep_$i.log 2>&1
  rc=$?; grep rows gpurun_out/sweep_$i.log; [ $rc -ne 0 ] && exit $rc
done
exit 0

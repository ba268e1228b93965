# r04 k: the whole GPU suite (kth-largest starting floor, graph-replayed embed forward, every parity test)
set -u
O=gpurun_out/r04k; mkdir -p $O
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
echo "gpu tests rc=$rc"; grep -E "passed|failed|error" $O/gpu_tests.log | tail -3
exit $rc

# round 3: euclidean scores in the 128-query FILTER: parity (euclidean, wide and query-group tests)
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r03ac
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_gpu_index.py -x -q --timeout 300 --timeout-method thread -k "wide or query_group or euclidean" > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/tests.log
exit $rc

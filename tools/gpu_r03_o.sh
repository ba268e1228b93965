# round 3: the 128-query FILTER (hr_wide.hip): parity tests, then the 10M batch sweep (new vs query groups)
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r03o
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_index.py -x -q --timeout 300 --timeout-method thread -k "wide or query_group" > $O/wide_tests.log 2>&1
rc=$?; echo "wide tests rc=$rc"; tail -5 $O/wide_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/sweep_batch.py --batches 64,128,256 --steps 60 > $O/sweep_wide.jsonl 2> $O/sweep_wide.err
rc=$?; echo "sweep rc=$rc"; cat $O/sweep_wide.jsonl; [ $rc -ne 0 ] && exit $rc
HIPRAG_WIDE_FILTER=0 timeout -k 10 300 python -u tools/sweep_batch.py --batches 128,256 --steps 60 > $O/sweep_groups.jsonl 2> $O/sweep_groups.err
rc=$?; echo "sweep (groups) rc=$rc"; cat $O/sweep_groups.jsonl

# round 3: row parts in the 128-query FILTER with every part refreshed at each refresh: parity, then FILTER time at
# 10M x 1024 B = 128 for k = 20 / 50 / 100 against query groups (HIPRAG_WIDE_PARTS=1)
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r03ae
mkdir -p $O
timeout -k 10 800 python -u -m pytest tests/test_gpu_index.py -x -v --timeout 300 --timeout-method thread -k "wide or query_group or euclidean" > $O/wide_tests.log 2>&1
rc=$?; echo "wide tests rc=$rc"; tail -3 $O/wide_tests.log; [ $rc -ne 0 ] && exit $rc
for k in 10 20 50 64 100; do
  for wp in 99 1; do
    HIPRAG_WIDE_PARTS=$wp timeout -k 10 200 python -u tools/diag_wide.py --reps 10 --k $k >> $O/diag.jsonl 2>> $O/diag.err || { echo "diag k=$k wp=$wp failed"; exit 1; }
    echo "parts<=$wp $(tail -1 $O/diag.jsonl)"
  done
done
exit 0

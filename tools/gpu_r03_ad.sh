# round 3: row parts in the 128-query FILTER (k 17..100 bf16 / f16, ..140 fp32) and fp32 rows actually dispatched to
# it: parity (wide / query-group / euclidean tests), then FILTER time at 10M x 1024 for k = 50 / 100 against query
# groups, and the fp32 batch sweep
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r03ad
mkdir -p $O
timeout -k 10 800 python -u -m pytest tests/test_gpu_index.py -x -v --timeout 300 --timeout-method thread -k "wide or query_group or euclidean" > $O/wide_tests.log 2>&1
rc=$?; echo "wide tests rc=$rc"; tail -3 $O/wide_tests.log; [ $rc -ne 0 ] && exit $rc
for k in 10 20 50 100; do
  for wf in 1 0; do
    HIPRAG_WIDE_FILTER=$wf timeout -k 10 200 python -u tools/diag_wide.py --reps 10 --k $k >> $O/diag.jsonl 2>> $O/diag.err || { echo "diag k=$k wf=$wf failed"; exit 1; }
    tail -1 $O/diag.jsonl
  done
done
timeout -k 10 400 python -u tools/sweep_batch.py --rows 10000000 --dim 1024 --dtype f32 --batches 64,128,256 --steps 30 > $O/sweep_10M_f32.jsonl 2> $O/sweep_10M_f32.err
rc=$?; echo "sweep 10M f32 rc=$rc"; cat $O/sweep_10M_f32.jsonl; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/sweep_batch.py --rows 10000000 --dim 1024 --batches 128,256 --k 50 --steps 30 > $O/sweep_10M_k50.jsonl 2> $O/sweep_10M_k50.err
rc=$?; echo "sweep 10M k50 rc=$rc"; cat $O/sweep_10M_k50.jsonl
exit 0

# round 3: DPP / ds_swizzle cross-lane reductions in the 128-query FILTER's refresh and epilogue (were ds_bpermute
# chains): parity, then FILTER time and candidates at 10M x 1024, B = 128, refresh every 1 / 2 / 4 rounds
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r03ah
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_index.py -x -q --timeout 300 --timeout-method thread -k "wide or query_group or euclidean" > $O/wide_tests.log 2>&1
rc=$?; echo "wide tests rc=$rc"; tail -2 $O/wide_tests.log; [ $rc -ne 0 ] && exit $rc
for k in 10 50; do
  for rt in 1 2 4; do
    HIPRAG_REFRESH=$rt timeout -k 10 200 python -u tools/diag_wide.py --reps 10 --k $k >> $O/diag.jsonl 2>> $O/diag.err || { echo "diag failed"; exit 1; }
    echo "rt=$rt $(tail -1 $O/diag.jsonl | cut -c1-330)"
  done
done
timeout -k 10 300 python -u tools/sweep_batch.py --batches 64,128,256 --steps 60 > $O/sweep.jsonl 2> $O/sweep.err
rc=$?; echo "sweep rc=$rc"; cat $O/sweep.jsonl
exit 0

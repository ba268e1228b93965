# round 3: eight-wave 128-query FILTER with refreshes every 2 rounds: parity, diagnostics, sweep
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r03t
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_index.py -x -q --timeout 300 --timeout-method thread -k "wide or query_group" > $O/wide_tests.log 2>&1
rc=$?; echo "wide tests rc=$rc"; tail -3 $O/wide_tests.log; [ $rc -ne 0 ] && exit $rc
for cfg in "HIPRAG_REFRESH=4" "HIPRAG_REFRESH=8"; do
  env $cfg timeout -k 10 200 python -u tools/diag_wide.py --reps 20 >> $O/diag.jsonl 2>> $O/diag.err || { echo "$cfg failed"; exit 1; }
  echo "$cfg: $(tail -1 $O/diag.jsonl)"
done
timeout -k 10 300 python -u tools/sweep_batch.py --batches 64,128,256 --steps 60 > $O/sweep_wide.jsonl 2> $O/sweep_wide.err
rc=$?; echo "sweep rc=$rc"; cat $O/sweep_wide.jsonl



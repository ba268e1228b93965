# round 3: eight-wave 128-query FILTER with two resident query windows: parity, diagnostics, sweep
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r03y
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_index.py -x -q --timeout 300 --timeout-method thread -k "wide or query_group" > $O/wide_tests.log 2>&1
rc=$?; echo "wide tests rc=$rc"; tail -3 $O/wide_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u tools/diag_wide.py --reps 20 > $O/diag.jsonl 2> $O/diag.err; echo "diag rc=$?"; cat $O/diag.jsonl
timeout -k 10 300 python -u tools/sweep_batch.py --batches 64,128,256 --steps 60 > $O/sweep_10M.jsonl 2> $O/sweep_10M.err
rc=$?; echo "sweep rc=$rc"; cat $O/sweep_10M.jsonl
timeout -k 10 300 python -u tools/sweep_batch.py --rows 1000000 --dim 768 --batches 128,256 --steps 100 > $O/sweep_c2.jsonl 2> $O/sweep_c2.err
rc=$?; echo "sweep c2 rc=$rc"; cat $O/sweep_c2.jsonl
exit 0

# round 3: the 128-query FILTER on fp32 rows: parity (wide + query-group tests), then 10M x 1024 f32 and 1M x 768 f32
# batch sweeps (fp32 rows are the store's default dtype)
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r03aa
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_gpu_index.py -x -q --timeout 300 --timeout-method thread -k "wide or query_group" > $O/wide_tests.log 2>&1
rc=$?; echo "wide tests rc=$rc"; tail -3 $O/wide_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/sweep_batch.py --rows 1000000 --dim 768 --dtype f32 --batches 64,128,256 --steps 60 > $O/sweep_c2_f32.jsonl 2> $O/sweep_c2_f32.err
rc=$?; echo "sweep c2 f32 rc=$rc"; cat $O/sweep_c2_f32.jsonl; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u tools/sweep_batch.py --rows 10000000 --dim 1024 --dtype f32 --batches 64,128,256 --steps 30 > $O/sweep_10M_f32.jsonl 2> $O/sweep_10M_f32.err
rc=$?; echo "sweep 10M f32 rc=$rc"; cat $O/sweep_10M_f32.jsonl; [ $rc -ne 0 ] && exit $rc
HIPRAG_WIDE_FILTER=0 timeout -k 10 400 python -u tools/sweep_batch.py --rows 10000000 --dim 1024 --dtype f32 --batches 128,256 --steps 30 > $O/sweep_10M_f32_old.jsonl 2> $O/sweep_10M_f32_old.err
rc=$?; echo "sweep 10M f32 (one group per pass) rc=$rc"; cat $O/sweep_10M_f32_old.jsonl
exit 0

# round 3: the pipelined group handle -- its GPU tests, then the single-process bench with 8 shards on
# the one GPU (10M rows: 8 x 1.25M) next to the single-handle 10M bench, the bf16-vs-fp32 recall test,
# and the row-part teams (k > 16): index tests, C3 parity at k = 100, benches at k = 45 / 100
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r03b
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_group.py tests/test_gpu_index.py -x -v --timeout 200 --timeout-method thread > $O/group_index_tests.log 2>&1
rc=$?; echo "group+index tests rc=$rc"; tail -3 $O/group_index_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u -m pytest tests/test_gpu_scale.py -x -v -s --timeout 280 --timeout-method thread -k "group_8_shards or recall_vs_fp32 or c3_10M_bf16" > $O/scale_tests.log 2>&1
rc=$?; echo "scale tests rc=$rc"; grep -a "C3 \|C2 1Mx768 bf16 store" $O/scale_tests.log; tail -2 $O/scale_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --single-process --gpus 8 --steps 100 --warmup 10 --no-cpu > $O/sp8.json 2> $O/sp8.err
rc=$?; echo "single-process x8 rc=$rc"; cat $O/sp8.json; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --steps 100 --warmup 10 --no-cpu > $O/one.json 2> $O/one.err
rc=$?; echo "single handle rc=$rc"; cat $O/one.json; [ $rc -ne 0 ] && exit $rc
for K in 45 100; do
timeout -k 10 300 python -u bench.py --steps 100 --warmup 10 --no-cpu --k $K > $O/k$K.json 2> $O/k$K.err
rc=$?; echo "k=$K rc=$rc"; cat $O/k$K.json; [ $rc -ne 0 ] && exit $rc
done
HIPRAG_PART_TEAMS=0 timeout -k 10 300 python -u bench.py --steps 100 --warmup 10 --no-cpu --k 100 > $O/k100_noteams.json 2> $O/k100_noteams.err
echo "k=100 teams off rc=$?"; cat $O/k100_noteams.json

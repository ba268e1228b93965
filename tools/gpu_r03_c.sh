# round 3: event-loop native launches of the store (GPU test + tools/bench_async.py A/B at 10M), row-part
# teams at k = 45 / 100 (A/B against contiguous parts), the 8-shards-on-one-GPU handle under stream
# variants, and the 1.25M shard step
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r03c
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_store.py -x -v --timeout 200 --timeout-method thread > $O/store_tests.log 2>&1
rc=$?; echo "store tests rc=$rc"; tail -3 $O/store_tests.log; [ $rc -ne 0 ] && exit $rc
for K in 45 100; do
timeout -k 10 300 python -u bench.py --steps 100 --warmup 10 --no-cpu --k $K > $O/k$K.json 2> $O/k$K.err
rc=$?; echo "k=$K rc=$rc"; cat $O/k$K.json; [ $rc -ne 0 ] && exit $rc
HIPRAG_PART_TEAMS=0 timeout -k 10 300 python -u bench.py --steps 100 --warmup 10 --no-cpu --k $K > $O/k${K}_noteams.json 2> $O/k${K}_noteams.err
rc=$?; echo "k=$K teams off rc=$rc"; cat $O/k${K}_noteams.json; [ $rc -ne 0 ] && exit $rc
done
timeout -k 10 300 python -u bench.py --rows 1250000 --steps 300 --warmup 10 --no-cpu > $O/shard1.25M.json 2> $O/shard1.25M.err
rc=$?; echo "1.25M rc=$rc"; cat $O/shard1.25M.json; [ $rc -ne 0 ] && exit $rc
for V in "" "HIPRAG_DUAL_SCAN=0" "HIPRAG_EARLY_SAMPLE=0"; do
env $V timeout -k 10 300 python -u bench.py --single-process --gpus 8 --steps 100 --warmup 10 --no-cpu > $O/sp8_$V.json 2> $O/sp8_$V.err
rc=$?; echo "sp8 [$V] rc=$rc"; cat $O/sp8_$V.json; [ $rc -ne 0 ] && exit $rc
done
timeout -k 10 600 python -u tools/bench_async.py --rows 10000000 --clients 1,16,64,256,1024 --max-batch 64,256 --native-async 1,0 --seconds 3 > $O/async_store_10M.jsonl 2> $O/async_store_10M.err
echo "bench_async rc=$?"; cat $O/async_store_10M.jsonl

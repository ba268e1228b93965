# round 3: packed (length-sorted) ingest batches; row-part early refresh default; quick parity
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r03h
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_embedder.py tests/test_gpu_index.py tests/test_gpu_scale.py -k "embedder or ingest or c4 or c3_10M or rowpart or part or topk" -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u tools/bench_ingest.py --chunks 100000 --preset bge-base --dtype bfloat16 > $O/ingest_100k_base.json 2> $O/ingest_100k_base.err
rc=$?; echo "ingest rc=$rc"; cat $O/ingest_100k_base.json; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats -T -d $O/prof_ingest -o run --output-format csv -- python3 tools/bench_ingest.py --chunks 20000 --preset bge-base --dtype bfloat16 --cpu-sample 8 > $O/ingest_prof.json 2> $O/ingest_prof.err
rc=$?; echo "ingest profile rc=$rc"; [ $rc -ne 0 ] && exit $rc
for K in 45 100; do
timeout -k 10 300 python -u bench.py --steps 100 --warmup 10 --no-cpu --k $K > $O/k$K.json 2> $O/k$K.err
rc=$?; echo "k=$K rc=$rc"; cut -c1-400 $O/k$K.json; [ $rc -ne 0 ] && exit $rc
done

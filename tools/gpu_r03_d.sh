# round 3: C4 ingest (bge-base shape, 100k chunks) and C5 rerank against the MFMA roof, each with a
# rocprofv3 kernel summary; the async store with gc.freeze 0/1; the 8-shards-on-one-GPU handle again
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r03d
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_index.py -x -q --timeout 200 --timeout-method thread > $O/index_tests.log 2>&1
rc=$?; echo "index tests rc=$rc"; tail -2 $O/index_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u tools/bench_ingest.py --chunks 100000 --preset bge-base --dtype bfloat16 > $O/ingest_100k_base.json 2> $O/ingest_100k_base.err
rc=$?; echo "ingest rc=$rc"; cat $O/ingest_100k_base.json; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats -T -d $O/prof_ingest -o run --output-format csv -- python3 tools/bench_ingest.py --chunks 20000 --preset bge-base --dtype bfloat16 --cpu-sample 8 > $O/ingest_prof.json 2> $O/ingest_prof.err
rc=$?; echo "ingest profile rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u tools/bench_rerank.py > $O/rerank.json 2> $O/rerank.err
rc=$?; echo "rerank rc=$rc"; cat $O/rerank.json; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats -T -d $O/prof_rerank -o run --output-format csv -- python3 tools/bench_rerank.py --no-exact --steps 5 > $O/rerank_prof.json 2> $O/rerank_prof.err
rc=$?; echo "rerank profile rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --single-process --gpus 8 --steps 100 --warmup 10 --no-cpu > $O/sp8.json 2> $O/sp8.err
rc=$?; echo "sp8 rc=$rc"; cat $O/sp8.json; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u tools/bench_async.py --rows 10000000 --clients 1,64,256,1024 --max-batch 64,256 --native-async 1 --gc-freeze 0,1 --seconds 3 > $O/async_store_10M.jsonl 2> $O/async_store_10M.err
echo "bench_async rc=$?"; cat $O/async_store_10M.jsonl

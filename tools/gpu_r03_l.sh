# round 3: co-located group shards on shared scan streams (A/B), ingest host profile
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r03l
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_group.py -x -q --timeout 240 --timeout-method thread > $O/group_tests.log 2>&1
rc=$?; echo "group tests rc=$rc"; tail -3 $O/group_tests.log; [ $rc -ne 0 ] && exit $rc
for V in 0 1 2 4; do
  HIPRAG_GROUP_SCAN_STREAMS=$V timeout -k 10 300 python -u bench.py --single-process --gpus 8 --steps 100 --warmup 10 --no-cpu > $O/sp8_gss$V.json 2> $O/sp8_gss$V.err
  rc=$?; echo "sp8 gss=$V rc=$rc"; cat $O/sp8_gss$V.json; [ $rc -ne 0 ] && exit $rc
done
timeout -k 10 400 python -u -m cProfile -o $O/ingest.pstats tools/bench_ingest.py --chunks 30000 --preset bge-base --dtype bfloat16 --cpu-sample 8 > $O/ingest_cprof.json 2> $O/ingest_cprof.err
rc=$?; echo "ingest cprofile rc=$rc"; cat $O/ingest_cprof.json; [ $rc -ne 0 ] && exit $rc
python -c "import pstats; s=pstats.Stats('$O/ingest.pstats'); s.sort_stats('tottime').print_stats(45); s.sort_stats('cumtime').print_stats(60)" > $O/ingest_pstats.txt
echo done
timeout -k 10 500 python -u -m pytest tests/test_gpu_embedder.py tests/test_gpu_reranker.py -x -q --timeout 300 --timeout-method thread > $O/emb_tests.log 2>&1
rc=$?; echo "embedder/reranker tests rc=$rc"; tail -3 $O/emb_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u tools/bench_ingest.py --chunks 100000 --preset bge-base --dtype bfloat16 > $O/ingest_100k_base.json 2> $O/ingest_100k_base.err
rc=$?; echo "ingest rc=$rc"; cat $O/ingest_100k_base.json; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u tools/bench_rerank.py > $O/rerank.json 2> $O/rerank.err
rc=$?; echo "rerank rc=$rc"; cat $O/rerank.json

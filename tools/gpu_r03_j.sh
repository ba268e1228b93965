# round 3: attention variants, the unpadded encoder (tests + C4 ingest + C5 rerank)
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r03j
mkdir -p $O
timeout -k 10 300 python -u tools/attn_micro.py > $O/attn_micro.jsonl 2> $O/attn_micro.err
echo "attn micro rc=$?"; cat $O/attn_micro.jsonl; tail -3 $O/attn_micro.err
timeout -k 10 500 python -u -m pytest tests/test_gpu_embedder.py tests/test_gpu_reranker.py tests/test_gpu_scale.py -k "embedder or reranker or ingest or c4 or unpadded or layernorm or k7 or k8 or topk" -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -a "PASS\|FAIL\|Error" $O/tests.log | tail -30; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u tools/bench_ingest.py --chunks 100000 --preset bge-base --dtype bfloat16 > $O/ingest_100k_base.json 2> $O/ingest_100k_base.err
rc=$?; echo "ingest rc=$rc"; cat $O/ingest_100k_base.json; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats -T -d $O/prof_ingest -o run --output-format csv -- python3 tools/bench_ingest.py --chunks 20000 --preset bge-base --dtype bfloat16 --cpu-sample 8 > $O/ingest_prof.json 2> $O/ingest_prof.err
rc=$?; echo "ingest profile rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u tools/bench_rerank.py > $O/rerank.json 2> $O/rerank.err
rc=$?; echo "rerank rc=$rc"; cat $O/rerank.json

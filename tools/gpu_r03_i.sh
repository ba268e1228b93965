# round 3: packed ingest with the asynchronous permutation upload
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r03i
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_embedder.py tests/test_gpu_scale.py -k "embedder or ingest or c4" -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u tools/bench_ingest.py --chunks 100000 --preset bge-base --dtype bfloat16 > $O/ingest_100k_base.json 2> $O/ingest_100k_base.err
rc=$?; echo "ingest rc=$rc"; cat $O/ingest_100k_base.json; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u tools/bench_ingest.py --chunks 100000 --preset bge-large --dtype bfloat16 > $O/ingest_100k_large.json 2> $O/ingest_100k_large.err
rc=$?; echo "ingest large rc=$rc"; cat $O/ingest_100k_large.json
timeout -k 10 300 python -u tools/attn_micro.py > $O/attn_micro.jsonl 2> $O/attn_micro.err
echo "attn micro rc=$?"; cat $O/attn_micro.jsonl; tail -3 $O/attn_micro.err

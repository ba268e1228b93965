# round 3: cached-id tokenizer + FLOP counting on the unpadded path (C4 ingest, C5 rerank), strided varlen
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r03k
mkdir -p $O
timeout -k 10 300 python -u tools/attn_micro.py > $O/attn_micro.jsonl 2> $O/attn_micro.err
echo "attn micro rc=$?"; cat $O/attn_micro.jsonl; tail -3 $O/attn_micro.err
timeout -k 10 600 python -u tools/bench_ingest.py --chunks 100000 --preset bge-base --dtype bfloat16 > $O/ingest_100k_base.json 2> $O/ingest_100k_base.err
rc=$?; echo "ingest rc=$rc"; cat $O/ingest_100k_base.json; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u tools/bench_rerank.py > $O/rerank.json 2> $O/rerank.err
rc=$?; echo "rerank rc=$rc"; cat $O/rerank.json

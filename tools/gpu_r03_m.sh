# round 3: co-located shards x SAMPLE size; rerank batch; kernel stats of the packed encoder (ingest, rerank)
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r03m
mkdir -p $O
for S in 2048 1024 512; do
  HIPRAG_SAMPLE_MIN=$S timeout -k 10 300 python -u bench.py --single-process --gpus 8 --steps 100 --warmup 10 --no-cpu > $O/sp8_smin$S.json 2> $O/sp8_smin$S.err
  rc=$?; echo "sp8 smin=$S rc=$rc"; cat $O/sp8_smin$S.json; [ $rc -ne 0 ] && exit $rc
done
timeout -k 10 600 python -u tools/bench_rerank.py --rerank-batch 1024 --no-exact > $O/rerank_b1024.json 2> $O/rerank_b1024.err
rc=$?; echo "rerank b1024 rc=$rc"; cat $O/rerank_b1024.json; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats -T -d $O/prof_rerank -o run --output-format csv -- python3 tools/bench_rerank.py --no-exact > $O/rerank_prof.json 2> $O/rerank_prof.err
rc=$?; echo "rerank profile rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats -T -d $O/prof_ingest -o run --output-format csv -- python3 tools/bench_ingest.py --chunks 20000 --preset bge-base --dtype bfloat16 --cpu-sample 8 > $O/ingest_prof.json 2> $O/ingest_prof.err
rc=$?; echo "ingest profile rc=$rc"; cat $O/ingest_prof.json

# round 3: pipelined GPU ingest (tests + 100k-chunk bench, with and without stage timing) and the
# 1.25M-shard knob sweep (tools/ab_env.sh, two alternating repeats per setting)
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r03f
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_embedder.py tests/test_gpu_scale.py -k "embedder or ingest or c4" -x -v --timeout 300 --timeout-method thread > $O/ingest_tests.log 2>&1
rc=$?; echo "ingest tests rc=$rc"; tail -3 $O/ingest_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u tools/bench_ingest.py --chunks 100000 --preset bge-base --dtype bfloat16 > $O/ingest_100k_base.json 2> $O/ingest_100k_base.err
rc=$?; echo "ingest rc=$rc"; cat $O/ingest_100k_base.json; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 bash tools/ab_env.sh "" "HIPRAG_TAIL_CUS=16" "HIPRAG_TAIL_CUS=48" "HIPRAG_DYN_PCT=5" "HIPRAG_DYN_PCT=20" "HIPRAG_DYN_CHUNK=4" > $O/ab_shard1.25M.log 2>&1
echo "ab rc=$?"; cat $O/ab_shard1.25M.log

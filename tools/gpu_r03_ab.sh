# round 3: the reference's call pattern through the store (10M x 1024 bf16) with the 128-query FILTER behind
# batches of up to 256 queries; with and without gc.freeze()
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r03ab
mkdir -p $O
timeout -k 10 600 python -u tools/bench_async.py --clients 64,256,1024 --max-batch 64,256 --gc-freeze 0,1 --seconds 3 > $O/async.jsonl 2> $O/async.err
rc=$?; echo "async rc=$rc"; cat $O/async.jsonl; tail -3 $O/async.err
exit $rc

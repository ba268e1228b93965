# round 3: GEMM ceiling at the encoder shapes; co-located shard defaults (tests + bench)
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r03n
mkdir -p $O
timeout -k 10 300 python -u tools/gemm_micro.py > $O/gemm_micro.jsonl 2> $O/gemm_micro.err
rc=$?; echo "gemm micro rc=$rc"; cat $O/gemm_micro.jsonl; [ $rc -ne 0 ] && exit $rc
timeout -k 10 500 python -u -m pytest tests/test_gpu_group.py "tests/test_gpu_scale.py::test_c3_group_8_shards_pipelined_vs_oracle" -x -q --timeout 400 --timeout-method thread > $O/group_tests.log 2>&1
rc=$?; echo "group tests rc=$rc"; tail -3 $O/group_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --single-process --gpus 8 --steps 100 --warmup 10 --no-cpu > $O/sp8.json 2> $O/sp8.err
rc=$?; echo "sp8 rc=$rc"; cat $O/sp8.json; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --steps 100 --warmup 10 --no-cpu > $O/single.json 2> $O/single.err
rc=$?; echo "single rc=$rc"; cat $O/single.json

# r04 a: RCCL world-size-1 exchange at C3, C3 parity (bf16 + fp32 default store), bench with/without the
# collective, kernel names under rocprofv3.  Each GPU step time-limited; the first failure ends the call.
set -u
O=gpurun_out/r04a; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_index.py -x -v -s -k "async_slots or query_group_edges or shard_search_f32" --timeout 120 --timeout-method thread > $O/idx.log 2>&1; rc=$?
echo "idx rc=$rc"; grep -E "PASS|FAIL|Error" $O/idx.log | tail -12; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u -m pytest tests/test_gpu_rccl.py -x -v -s --timeout 300 --timeout-method thread > $O/rccl.log 2>&1; rc=$?
echo "rccl rc=$rc"; tail -5 $O/rccl.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 700 python -u -m pytest tests/test_gpu_scale.py -x -v -s -k "c3_10M" --timeout 600 --timeout-method thread > $O/c3.log 2>&1; rc=$?
echo "c3 rc=$rc"; grep -E "C3 10M|passed|failed" $O/c3.log | tail -12; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --steps 200 --warmup 10 --no-cpu > $O/bench.json 2> $O/bench.err; rc=$?
echo "bench rc=$rc"; cat $O/bench.json; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --steps 200 --warmup 10 --no-cpu --collective > $O/bench_coll.json 2> $O/bench_coll.err; rc=$?
echo "bench coll rc=$rc"; cat $O/bench_coll.json; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --rows 1250000 --steps 400 --warmup 10 --no-cpu > $O/bench_shard.json 2> $O/bench_shard.err; rc=$?
echo "bench shard rc=$rc"; cat $O/bench_shard.json; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d $O/kt -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu > $O/kt.log 2>&1; rc=$?
echo "kt rc=$rc"; [ $rc -ne 0 ] && exit $rc
python3 tools/summarize_profile.py $O r04a_10Mx1024_b64_probe 20480000000 > $O/summary.log 2>&1; grep -E "filter_kernels|filter_ms|launches|achieved" $O/summary.log

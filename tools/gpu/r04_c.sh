# r04 c: persist + dealing tests, 1.25M A/B, 10M regression check, the default bench (CPU legs, recall 64+64, GPU
# embed leg), the async store without an application gc.freeze
set -u
O=gpurun_out/r04c; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_persist.py tests/test_gpu_index.py -x -v -s -k "persist or exactly_once or async_slots or wide_filter" --timeout 240 --timeout-method thread > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "PASS|FAIL|Error" $O/tests.log | tail -12; [ $rc -ne 0 ] && exit $rc
for m in 1 0 1 0; do
  timeout -k 10 200 python -u bench.py --rows 1250000 --steps 400 --warmup 10 --no-cpu --persist $m > $O/shard_p$m.json 2> $O/shard_p$m.err; rc=$?
  echo "shard persist=$m rc=$rc"; [ $rc -ne 0 ] && { tail -5 $O/shard_p$m.err; exit $rc; }
  python3 -c "import json;d=json.load(open('$O/shard_p$m.json'));r=d['roofline'];print(d['value'],d['ms_per_step'],r['avg_launch_ms'],r['frac'],r['kernel'][:20])"
done
timeout -k 10 300 python -u bench.py --steps 200 --warmup 10 --no-cpu > $O/10M.json 2> $O/10M.err; rc=$?
echo "10M rc=$rc"; [ $rc -ne 0 ] && { tail -5 $O/10M.err; exit $rc; }
python3 -c "import json;d=json.load(open('$O/10M.json'));r=d['roofline'];print(d['value'],d['ms_per_step'],r['avg_launch_ms'],r['frac'],r['kernel'][:20])"
timeout -k 10 300 python -u bench.py --steps 200 --warmup 10 --no-cpu --persist 2 > $O/10M_p2.json 2> $O/10M_p2.err; rc=$?
echo "10M p2 rc=$rc"; [ $rc -ne 0 ] && { tail -5 $O/10M_p2.err; exit $rc; }
python3 -c "import json;d=json.load(open('$O/10M_p2.json'));r=d['roofline'];print(d['value'],d['ms_per_step'],r['avg_launch_ms'],r['frac'],r['kernel'][:20])"
timeout -k 10 600 python -u bench.py > $O/default.json 2> $O/default.err; rc=$?
echo "default bench rc=$rc"; [ $rc -ne 0 ] && { tail -5 $O/default.err; exit $rc; }
python3 -c "import json;d=json.load(open('$O/default.json'));print(d['value'],d.get('recall_at_10_vs_fp32'),d.get('gpu_embed_plus_search'),d['cpu_baseline'].get('value'))"
timeout -k 10 400 python -u tools/bench_async.py --rows 10000000 --clients 256,1024 --max-batch 64,256 --seconds 3 --gc-freeze 0 > $O/async.jsonl 2> $O/async.err; rc=$?
echo "async rc=$rc"; cat $O/async.jsonl

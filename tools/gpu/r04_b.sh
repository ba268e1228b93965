# r04 b: persistent FILTER parity, then the 1.25M-row shard A/B (persist on / off, alternating), then the suites it touches
set -u
O=gpurun_out/r04b; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_persist.py -x -v -s --timeout 240 --timeout-method thread > $O/persist.log 2>&1; rc=$?
echo "persist tests rc=$rc"; grep -E "PASS|FAIL|Error|error" $O/persist.log | tail -15; [ $rc -ne 0 ] && exit $rc
for m in 1 0 1 0; do
  timeout -k 10 200 python -u bench.py --rows 1250000 --steps 400 --warmup 10 --no-cpu --persist $m > $O/shard_p$m.json 2> $O/shard_p$m.err; rc=$?
  echo "shard persist=$m rc=$rc"; [ $rc -ne 0 ] && { tail -5 $O/shard_p$m.err; exit $rc; }
  python3 -c "import json;d=json.load(open('$O/shard_p$m.json'));r=d['roofline'];print(d['value'],d['ms_per_step'],r['avg_launch_ms'],r['frac'],r['kernel'][:20])"
done
timeout -k 10 300 python -u bench.py --steps 100 --warmup 10 --no-cpu --persist 2 > $O/10M_p2.json 2> $O/10M_p2.err; rc=$?
echo "10M persist=2 rc=$rc"; [ $rc -ne 0 ] && { tail -5 $O/10M_p2.err; exit $rc; }
python3 -c "import json;d=json.load(open('$O/10M_p2.json'));r=d['roofline'];print(d['value'],d['ms_per_step'],r['avg_launch_ms'],r['frac'],r['kernel'][:20])"
timeout -k 10 900 python -u -m pytest tests/test_gpu_index.py tests/test_gpu_dist.py -x -q --timeout 240 --timeout-method thread > $O/idx.log 2>&1; rc=$?
echo "index+dist rc=$rc"; tail -3 $O/idx.log

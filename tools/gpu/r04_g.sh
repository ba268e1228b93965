# r04 g: persistent FILTER with write-through candidate stores (no per-batch release fence): parity, then
# per-batch launches vs the persistent FILTER over shard sizes
set -u
O=gpurun_out/r04g; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_persist.py > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "passed|failed|error" $O/tests.log | tail -3; [ $rc -ne 0 ] && exit $rc
run() {  # tag, command...
  tag=$1; shift
  timeout -k 10 240 "$@" --no-cpu --no-embed --steps 60 --warmup 5 > $O/$tag.json 2> $O/$tag.err; rc=$?
  echo "$tag rc=$rc"; [ $rc -ne 0 ] && { tail -5 $O/$tag.err; exit $rc; }
  python3 -c "import json,sys;d=json.load(open('$O/$tag.json'));r=d['roofline'];print(d['value'],d['ms_per_step'],r['avg_launch_ms'],r['frac'],d.get('persist_timeline'))"
}
for rep in 1 2; do
  run r1250000_p0_$rep python3 bench.py --rows 1250000 --persist 0
  run r1250000_p1_$rep python3 bench.py --rows 1250000 --persist 1
done
for rows in 2500000 5000000; do
  run r${rows}_p0 python3 bench.py --rows $rows --persist 0
  run r${rows}_p1 python3 bench.py --rows $rows --persist 1
done
echo done

# r04 v: direct RCCL with every call on the tail stream (fallback gather and broadcast included): RCCL + dist parity
# tests, then the collective benches
set -u
O=gpurun_out/r04v; mkdir -p $O
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_rccl.py tests/test_gpu_dist.py > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "passed|failed|error" $O/tests.log | tail -3; [ $rc -ne 0 ] && exit $rc
run() {  # tag, command...
  tag=$1; shift
  timeout -k 10 240 "$@" --no-cpu --no-embed > $O/$tag.json 2> $O/$tag.err; rc=$?
  echo "$tag rc=$rc"; [ $rc -ne 0 ] && { tail -5 $O/$tag.err; exit $rc; }
  python3 -c "import json,sys;d=json.load(open('$O/$tag.json'));r=d['roofline'];print(d['value'],d['ms_per_step'],d.get('host_ms_per_step'),r['avg_launch_ms'],d['config']['exchange'])"
}
run s125_rccl python3 bench.py --rows 1250000 --steps 200 --warmup 10 --collective
run m10_rccl python3 bench.py --steps 100 --warmup 10 --collective
run m10_local python3 bench.py --steps 100 --warmup 10
echo done

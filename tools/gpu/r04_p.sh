# r04 p: 1024-tile SAMPLE floor (this tree) vs 2048 (ab/libhiprag_s2k.so) over shard sizes, alternating; then the
# index / persist parity tests on this tree
set -u
O=gpurun_out/r04p; mkdir -p $O
run() {  # tag, command...
  tag=$1; shift
  timeout -k 10 240 "$@" --no-cpu --no-embed > $O/$tag.json 2> $O/$tag.err; rc=$?
  echo "$tag rc=$rc"; [ $rc -ne 0 ] && { tail -5 $O/$tag.err; exit $rc; }
  python3 -c "import json,sys;d=json.load(open('$O/$tag.json'));r=d['roofline'];print(d['value'],d['ms_per_step'],r['avg_launch_ms'],r['frac'],r.get('guard_fallback_queries'))"
}
for rep in 1 2; do
  run c2_s1k_$rep python3 bench.py --rows 1000000 --dim 768 --steps 100 --warmup 10
  HIPRAG_LIB_OVERRIDE=ab/libhiprag_s2k.so run c2_s2k_$rep python3 bench.py --rows 1000000 --dim 768 --steps 100 --warmup 10
  run r25_s1k_$rep python3 bench.py --rows 2500000 --steps 100 --warmup 10
  HIPRAG_LIB_OVERRIDE=ab/libhiprag_s2k.so run r25_s2k_$rep python3 bench.py --rows 2500000 --steps 100 --warmup 10
  run r5_s1k_$rep python3 bench.py --rows 5000000 --steps 60 --warmup 5
  HIPRAG_LIB_OVERRIDE=ab/libhiprag_s2k.so run r5_s2k_$rep python3 bench.py --rows 5000000 --steps 60 --warmup 5
  run s125_s1k_$rep python3 bench.py --rows 1250000 --steps 200 --warmup 10
  HIPRAG_LIB_OVERRIDE=ab/libhiprag_s2k.so run s125_s2k_$rep python3 bench.py --rows 1250000 --steps 200 --warmup 10
done
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_index.py tests/test_gpu_persist.py tests/test_gpu_scale.py > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 $O/tests.log
exit $rc

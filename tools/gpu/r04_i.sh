# r04 i: k_scan's threshold refresh as DPP + ds_swizzle (this tree) vs the ds_bpermute chain (ab/libhiprag_base.so),
# alternating on one box; then the GPU parity tests of the scan paths that refresh
set -u
O=gpurun_out/r04i; mkdir -p $O
export TMPDIR=/tmp
run() {  # tag, command...
  tag=$1; shift
  timeout -k 10 240 "$@" --no-cpu --no-embed > $O/$tag.json 2> $O/$tag.err; rc=$?
  echo "$tag rc=$rc"; [ $rc -ne 0 ] && { tail -5 $O/$tag.err; exit $rc; }
  python3 -c "import json,sys;d=json.load(open('$O/$tag.json'));r=d['roofline'];print(d['value'],d['ms_per_step'],r['avg_launch_ms'],r['frac'])"
}
for rep in 1 2 3; do
  run m10_dpp_$rep python3 bench.py --steps 100 --warmup 10
  HIPRAG_LIB_OVERRIDE=ab/libhiprag_base.so run m10_base_$rep python3 bench.py --steps 100 --warmup 10
  run s125_dpp_$rep python3 bench.py --rows 1250000 --steps 200 --warmup 10
  HIPRAG_LIB_OVERRIDE=ab/libhiprag_base.so run s125_base_$rep python3 bench.py --rows 1250000 --steps 200 --warmup 10
done
for rep in 1 2; do
  run k100_dpp_$rep python3 bench.py --k 100 --steps 60 --warmup 5
  HIPRAG_LIB_OVERRIDE=ab/libhiprag_base.so run k100_base_$rep python3 bench.py --k 100 --steps 60 --warmup 5
done
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_index.py tests/test_gpu_persist.py > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 $O/tests.log
exit $rc

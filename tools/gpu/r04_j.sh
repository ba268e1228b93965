# r04 j: FILTER thresholds started at the kj-th largest sampled group maximum (k_floor_kth, this tree) vs the smallest
# (ab/libhiprag_base.so), alternating on one box, with the timed region's guard fallbacks
set -u
O=gpurun_out/r04j; mkdir -p $O
export TMPDIR=/tmp
run() {  # tag, command...
  tag=$1; shift
  timeout -k 10 240 "$@" --no-cpu --no-embed > $O/$tag.json 2> $O/$tag.err; rc=$?
  echo "$tag rc=$rc"; [ $rc -ne 0 ] && { tail -5 $O/$tag.err; exit $rc; }
  python3 -c "import json,sys;d=json.load(open('$O/$tag.json'));r=d['roofline'];print(d['value'],d['ms_per_step'],r['avg_launch_ms'],r['frac'],r.get('guard_fallback_queries'))"
}
for rep in 1 2 3; do
  run m10_kth_$rep python3 bench.py --steps 100 --warmup 10
  HIPRAG_LIB_OVERRIDE=ab/libhiprag_base.so run m10_base_$rep python3 bench.py --steps 100 --warmup 10
  run s125_kth_$rep python3 bench.py --rows 1250000 --steps 200 --warmup 10
  HIPRAG_LIB_OVERRIDE=ab/libhiprag_base.so run s125_base_$rep python3 bench.py --rows 1250000 --steps 200 --warmup 10
done
for rep in 1 2; do
  run b128_kth_$rep python3 bench.py --batch 128 --steps 60 --warmup 5
  HIPRAG_LIB_OVERRIDE=ab/libhiprag_base.so run b128_base_$rep python3 bench.py --batch 128 --steps 60 --warmup 5
done
run s5m_kth python3 bench.py --rows 5000000 --steps 60 --warmup 5
HIPRAG_LIB_OVERRIDE=ab/libhiprag_base.so run s5m_base python3 bench.py --rows 5000000 --steps 60 --warmup 5
run c2_kth python3 bench.py --rows 1000000 --dim 768 --steps 100 --warmup 10
HIPRAG_LIB_OVERRIDE=ab/libhiprag_base.so run c2_base python3 bench.py --rows 1000000 --dim 768 --steps 100 --warmup 10
echo done

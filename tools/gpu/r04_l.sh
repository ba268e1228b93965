# r04 l: k_scan refreshes staggered over the waves (this tree) vs all waves every 4th tile (ab/libhiprag_kth.so),
# alternating on one box
set -u
O=gpurun_out/r04l; mkdir -p $O
export TMPDIR=/tmp
run() {  # tag, command...
  tag=$1; shift
  timeout -k 10 240 "$@" --no-cpu --no-embed > $O/$tag.json 2> $O/$tag.err; rc=$?
  echo "$tag rc=$rc"; [ $rc -ne 0 ] && { tail -5 $O/$tag.err; exit $rc; }
  python3 -c "import json,sys;d=json.load(open('$O/$tag.json'));r=d['roofline'];print(d['value'],d['ms_per_step'],r['avg_launch_ms'],r['frac'],r.get('guard_fallback_queries'))"
}
for rep in 1 2 3; do
  run m10_stag_$rep python3 bench.py --steps 100 --warmup 10
  HIPRAG_LIB_OVERRIDE=ab/libhiprag_kth.so run m10_base_$rep python3 bench.py --steps 100 --warmup 10
  run s125_stag_$rep python3 bench.py --rows 1250000 --steps 200 --warmup 10
  HIPRAG_LIB_OVERRIDE=ab/libhiprag_kth.so run s125_base_$rep python3 bench.py --rows 1250000 --steps 200 --warmup 10
done
for rep in 1 2; do
  run k100_stag_$rep python3 bench.py --k 100 --steps 60 --warmup 5
  HIPRAG_LIB_OVERRIDE=ab/libhiprag_kth.so run k100_base_$rep python3 bench.py --k 100 --steps 60 --warmup 5
  run c2_stag_$rep python3 bench.py --rows 1000000 --dim 768 --steps 100 --warmup 10
  HIPRAG_LIB_OVERRIDE=ab/libhiprag_kth.so run c2_base_$rep python3 bench.py --rows 1000000 --dim 768 --steps 100 --warmup 10
done
echo done

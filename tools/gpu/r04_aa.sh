# r04 aa: the 128-query FILTER's refresh cadence -- every 4 rounds (this tree) vs 8 / 16 (ab/) -- B = 128 and 256
set -u
O=gpurun_out/r04aa; mkdir -p $O
run() {  # tag, command...
  tag=$1; shift
  timeout -k 10 240 "$@" --no-cpu --no-embed > $O/$tag.json 2> $O/$tag.err; rc=$?
  echo "$tag rc=$rc"; [ $rc -ne 0 ] && { tail -5 $O/$tag.err; exit $rc; }
  python3 -c "import json,sys;d=json.load(open('$O/$tag.json'));r=d['roofline'];print(d['value'],d['ms_per_step'],r['avg_launch_ms'],r['frac'],r.get('guard_fallback_queries'))"
}
for rep in 1 2; do
  run b128_rt4_$rep python3 bench.py --batch 128 --steps 60 --warmup 5
  HIPRAG_LIB_OVERRIDE=ab/libhiprag_w8.so run b128_rt8_$rep python3 bench.py --batch 128 --steps 60 --warmup 5
  HIPRAG_LIB_OVERRIDE=ab/libhiprag_w16.so run b128_rt16_$rep python3 bench.py --batch 128 --steps 60 --warmup 5
done
run b256_rt4 python3 bench.py --batch 256 --steps 30 --warmup 3
HIPRAG_LIB_OVERRIDE=ab/libhiprag_w8.so run b256_rt8 python3 bench.py --batch 256 --steps 30 --warmup 3
HIPRAG_LIB_OVERRIDE=ab/libhiprag_w16.so run b256_rt16 python3 bench.py --batch 256 --steps 30 --warmup 3
echo done

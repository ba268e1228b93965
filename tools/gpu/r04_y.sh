# r04 y: SAMPLE of n/256 tiles on large shards (ab/libhiprag_s256.so) vs n/128 (this tree), 10M rows and k = 100
set -u
O=gpurun_out/r04y; mkdir -p $O
run() {  # tag, command...
  tag=$1; shift
  timeout -k 10 240 "$@" --no-cpu --no-embed > $O/$tag.json 2> $O/$tag.err; rc=$?
  echo "$tag rc=$rc"; [ $rc -ne 0 ] && { tail -5 $O/$tag.err; exit $rc; }
  python3 -c "import json,sys;d=json.load(open('$O/$tag.json'));r=d['roofline'];print(d['value'],d['ms_per_step'],r['avg_launch_ms'],r['frac'],r.get('guard_fallback_queries'))"
}
for rep in 1 2 3; do
  run m10_s128_$rep python3 bench.py --steps 100 --warmup 10
  HIPRAG_LIB_OVERRIDE=ab/libhiprag_s256.so run m10_s256_$rep python3 bench.py --steps 100 --warmup 10
done
run k100_s128 python3 bench.py --k 100 --steps 60 --warmup 5
HIPRAG_LIB_OVERRIDE=ab/libhiprag_s256.so run k100_s256 python3 bench.py --k 100 --steps 60 --warmup 5
echo done

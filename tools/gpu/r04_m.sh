# r04 m: conditional stagger (large shards only) vs the kth build, then the round's final runs (r04_final.sh)
set -u
O=gpurun_out/r04m; mkdir -p $O
run() {  # tag, command...
  tag=$1; shift
  timeout -k 10 240 "$@" --no-cpu --no-embed > $O/$tag.json 2> $O/$tag.err; rc=$?
  echo "$tag rc=$rc"; [ $rc -ne 0 ] && { tail -5 $O/$tag.err; exit $rc; }
  python3 -c "import json,sys;d=json.load(open('$O/$tag.json'));r=d['roofline'];print(d['value'],d['ms_per_step'],r['avg_launch_ms'],r['frac'],r.get('guard_fallback_queries'))"
}
for rep in 1 2; do
  run m10_cond_$rep python3 bench.py --steps 100 --warmup 10
  HIPRAG_LIB_OVERRIDE=ab/libhiprag_kth.so run m10_base_$rep python3 bench.py --steps 100 --warmup 10
  run s125_cond_$rep python3 bench.py --rows 1250000 --steps 200 --warmup 10
  HIPRAG_LIB_OVERRIDE=ab/libhiprag_kth.so run s125_base_$rep python3 bench.py --rows 1250000 --steps 200 --warmup 10
done
bash tools/gpu/r04_final.sh

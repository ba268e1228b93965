# r04 n: refresh cadence on large shards (staggered): every 4 tiles (this tree) vs 2 / 8, and the stagger offset by
# workgroup too -- 10M rows, alternating on one box
set -u
O=gpurun_out/r04n; mkdir -p $O
run() {  # tag, command...
  tag=$1; shift
  timeout -k 10 240 "$@" --no-cpu --no-embed > $O/$tag.json 2> $O/$tag.err; rc=$?
  echo "$tag rc=$rc"; [ $rc -ne 0 ] && { tail -5 $O/$tag.err; exit $rc; }
  python3 -c "import json,sys;d=json.load(open('$O/$tag.json'));r=d['roofline'];print(d['value'],d['ms_per_step'],r['avg_launch_ms'],r['frac'],r.get('guard_fallback_queries'))"
}
for rep in 1 2; do
  run m10_rt4_$rep python3 bench.py --steps 100 --warmup 10
  for v in rt2 rt8 wgst; do
    HIPRAG_LIB_OVERRIDE=ab/libhiprag_$v.so run m10_${v}_$rep python3 bench.py --steps 100 --warmup 10
  done
done
for v in rt4 rt2 rt8 wgst; do
  if [ $v = rt4 ]; then run k100_$v python3 bench.py --k 100 --steps 60 --warmup 5
  else HIPRAG_LIB_OVERRIDE=ab/libhiprag_$v.so run k100_$v python3 bench.py --k 100 --steps 60 --warmup 5; fi
done
echo done

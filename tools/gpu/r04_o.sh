# r04 o: small-shard SAMPLE size (1024 / 3072 tiles vs 2048) and refresh cadence (every 2 tiles vs 4) with the
# kth-largest starting floor -- 1.25M rows and C2 (1M x 768), alternating on one box
set -u
O=gpurun_out/r04o; mkdir -p $O
run() {  # tag, command...
  tag=$1; shift
  timeout -k 10 240 "$@" --no-cpu --no-embed > $O/$tag.json 2> $O/$tag.err; rc=$?
  echo "$tag rc=$rc"; [ $rc -ne 0 ] && { tail -5 $O/$tag.err; exit $rc; }
  python3 -c "import json,sys;d=json.load(open('$O/$tag.json'));r=d['roofline'];print(d['value'],d['ms_per_step'],r['avg_launch_ms'],r['frac'],r.get('guard_fallback_queries'))"
}
for rep in 1 2; do
  run s125_cur_$rep python3 bench.py --rows 1250000 --steps 200 --warmup 10
  for v in s1k s3k rt2s; do
    HIPRAG_LIB_OVERRIDE=ab/libhiprag_$v.so run s125_${v}_$rep python3 bench.py --rows 1250000 --steps 200 --warmup 10
  done
done
run c2_cur python3 bench.py --rows 1000000 --dim 768 --steps 100 --warmup 10
for v in s1k s3k rt2s; do
  HIPRAG_LIB_OVERRIDE=ab/libhiprag_$v.so run c2_$v python3 bench.py --rows 1000000 --dim 768 --steps 100 --warmup 10
done
echo done

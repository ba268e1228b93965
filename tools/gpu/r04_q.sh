# r04 q: the kj-th largest starting floor with row parts (k > 16; this tree) vs without (ab/libhiprag_noparts.so),
# alternating; then the whole GPU suite on this tree
set -u
O=gpurun_out/r04q; mkdir -p $O
run() {  # tag, command...
  tag=$1; shift
  timeout -k 10 240 "$@" --no-cpu --no-embed > $O/$tag.json 2> $O/$tag.err; rc=$?
  echo "$tag rc=$rc"; [ $rc -ne 0 ] && { tail -5 $O/$tag.err; exit $rc; }
  python3 -c "import json,sys;d=json.load(open('$O/$tag.json'));r=d['roofline'];print(d['value'],d['ms_per_step'],r['avg_launch_ms'],r['frac'],r.get('guard_fallback_queries'))"
}
for rep in 1 2; do
  run k100_parts_$rep python3 bench.py --k 100 --steps 60 --warmup 5
  HIPRAG_LIB_OVERRIDE=ab/libhiprag_noparts.so run k100_base_$rep python3 bench.py --k 100 --steps 60 --warmup 5
  run k45_parts_$rep python3 bench.py --k 45 --steps 60 --warmup 5
  HIPRAG_LIB_OVERRIDE=ab/libhiprag_noparts.so run k45_base_$rep python3 bench.py --k 45 --steps 60 --warmup 5
  run k100s_parts_$rep python3 bench.py --rows 1250000 --k 100 --steps 100 --warmup 10
  HIPRAG_LIB_OVERRIDE=ab/libhiprag_noparts.so run k100s_base_$rep python3 bench.py --rows 1250000 --k 100 --steps 100 --warmup 10
done
run r5_cur python3 bench.py --rows 5000000 --steps 60 --warmup 5
run c2_cur python3 bench.py --rows 1000000 --dim 768 --steps 100 --warmup 10
bash tools/gpu/r04_k.sh

# r04 z: SAMPLE n/512 (ab/libhiprag_s512.so) vs n/256 (this tree) at 10M rows, then the whole GPU suite on this tree
set -u
O=gpurun_out/r04z; mkdir -p $O
run() {  # tag, command...
  tag=$1; shift
  timeout -k 10 240 "$@" --no-cpu --no-embed > $O/$tag.json 2> $O/$tag.err; rc=$?
  echo "$tag rc=$rc"; [ $rc -ne 0 ] && { tail -5 $O/$tag.err; exit $rc; }
  python3 -c "import json,sys;d=json.load(open('$O/$tag.json'));r=d['roofline'];print(d['value'],d['ms_per_step'],r['avg_launch_ms'],r['frac'],r.get('guard_fallback_queries'))"
}
for rep in 1 2 3; do
  run m10_s256_$rep python3 bench.py --steps 100 --warmup 10
  HIPRAG_LIB_OVERRIDE=ab/libhiprag_s512.so run m10_s512_$rep python3 bench.py --steps 100 --warmup 10
done
bash tools/gpu/r04_k.sh

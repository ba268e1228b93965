# r04 r: the 1.25M-row shard (the G = 8 per-rank step) through the RCCL exchange at world size 1 vs the local copy
set -u
O=gpurun_out/r04r; mkdir -p $O
run() {  # tag, command...
  tag=$1; shift
  timeout -k 10 240 "$@" --no-cpu --no-embed > $O/$tag.json 2> $O/$tag.err; rc=$?
  echo "$tag rc=$rc"; [ $rc -ne 0 ] && { tail -5 $O/$tag.err; exit $rc; }
  python3 -c "import json,sys;d=json.load(open('$O/$tag.json'));r=d['roofline'];print(d['value'],d['ms_per_step'],r['avg_launch_ms'],r['frac'],d['config']['parallelism'])"
}
for rep in 1 2; do
  run s125_rccl_$rep python3 bench.py --rows 1250000 --steps 200 --warmup 10 --collective
  run s125_local_$rep python3 bench.py --rows 1250000 --steps 200 --warmup 10
  run r25_rccl_$rep python3 bench.py --rows 2500000 --steps 100 --warmup 10 --collective
  run r5_rccl_$rep python3 bench.py --rows 5000000 --steps 60 --warmup 5 --collective
done
echo done

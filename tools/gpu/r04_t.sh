# r04 t: pipeline depth (batches in flight per rank) 2 vs 3, with and without the RCCL exchange, 1.25M rows
set -u
O=gpurun_out/r04t; mkdir -p $O
run() {  # tag, command...
  tag=$1; shift
  timeout -k 10 240 "$@" --no-cpu --no-embed > $O/$tag.json 2> $O/$tag.err; rc=$?
  echo "$tag rc=$rc"; [ $rc -ne 0 ] && { tail -5 $O/$tag.err; exit $rc; }
  python3 -c "import json,sys;d=json.load(open('$O/$tag.json'));r=d['roofline'];print(d['value'],d['ms_per_step'],d.get('host_ms_per_step'),r['avg_launch_ms'],d['config']['parallelism'])"
}
for rep in 1 2; do
  run s125_rccl_d2_$rep python3 bench.py --rows 1250000 --steps 200 --warmup 10 --collective --depth 2
  run s125_rccl_d3_$rep python3 bench.py --rows 1250000 --steps 200 --warmup 10 --collective --depth 3
  run s125_local_d2_$rep python3 bench.py --rows 1250000 --steps 200 --warmup 10 --depth 2
  run s125_local_d3_$rep python3 bench.py --rows 1250000 --steps 200 --warmup 10 --depth 3
done
run m10_local_d3 python3 bench.py --steps 100 --warmup 10 --depth 3
run m10_local_d2 python3 bench.py --steps 100 --warmup 10 --depth 2
run r5_rccl_d3 python3 bench.py --rows 5000000 --steps 60 --warmup 5 --collective --depth 3
echo done

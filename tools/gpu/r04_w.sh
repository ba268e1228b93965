# r04 w: direct RCCL at 10M rows -- RCCL's channel count (NCCL_MAX_NCHANNELS: CUs its kernels take beside the
# FILTER) 2 / 4 vs the default, and the local copy
set -u
O=gpurun_out/r04w; mkdir -p $O
run() {  # tag, command...
  tag=$1; shift
  timeout -k 10 240 "$@" --no-cpu --no-embed > $O/$tag.json 2> $O/$tag.err; rc=$?
  echo "$tag rc=$rc"; [ $rc -ne 0 ] && { tail -5 $O/$tag.err; exit $rc; }
  python3 -c "import json,sys;d=json.load(open('$O/$tag.json'));r=d['roofline'];print(d['value'],d['ms_per_step'],d.get('host_ms_per_step'),r['avg_launch_ms'])"
}
for rep in 1 2; do
  run m10_def_$rep python3 bench.py --steps 100 --warmup 10 --collective
  NCCL_MAX_NCHANNELS=2 run m10_ch2_$rep python3 bench.py --steps 100 --warmup 10 --collective
  NCCL_MAX_NCHANNELS=4 run m10_ch4_$rep python3 bench.py --steps 100 --warmup 10 --collective
  run m10_local_$rep python3 bench.py --steps 100 --warmup 10
done
NCCL_MAX_NCHANNELS=2 run s125_ch2 python3 bench.py --rows 1250000 --steps 200 --warmup 10 --collective
echo done

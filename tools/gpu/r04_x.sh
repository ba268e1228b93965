# r04 x: kernel traces of C2 (1M x 768) and the 1.25M shard with the final code, for their per-step timelines;
# then the 1.25M profile passes (summary regenerated with the 1024-tile SAMPLE)
set -u
export TMPDIR=/tmp
O=gpurun_out/r04x; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d $O/c2 -o run --output-format csv -- python3 bench.py --rows 1000000 --dim 768 --steps 100 --warmup 10 --no-cpu --no-embed > $O/c2.log 2>&1; rc=$?
echo "c2 trace rc=$rc"; [ $rc -ne 0 ] && exit $rc
bash tools/profile.sh r04final2_shard1.25M --rows 1250000 --steps 200 --warmup 10 --no-cpu --no-embed || exit $?
echo done

# r04 final: smoke, the driver's bench command (full: CPU baseline, recall, GPU embed leg), then rocprofv3 of the
# headline bench and of the 1.25M-row shard (kernel trace + PMC passes, tools/profile.sh)
set -u
O=gpurun_out/r04final3; mkdir -p $O
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?
echo "smoke rc=$rc"; tail -2 $O/smoke.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u bench.py > $O/bench_10M.json 2> $O/bench_10M.err; rc=$?
echo "bench rc=$rc"; tail -c 600 $O/bench_10M.json; [ $rc -ne 0 ] && { tail -5 $O/bench_10M.err; exit $rc; }
bash tools/profile.sh r04final3_10M --steps 20 --warmup 5 --no-cpu || exit $?
bash tools/profile.sh r04final3_shard1.25M --rows 1250000 --steps 200 --warmup 10 --no-cpu || exit $?
echo done

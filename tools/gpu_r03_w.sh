# round 3: the 128-query FILTER (final): GPU suite, batch sweeps at 10M x 1024 and 1M x 768, bench lines at
# B = 128 / 256, rocprofv3 of the B = 128 and B = 256 bench commands (kernel trace + stats, FETCH_SIZE, WRITE_SIZE)
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r03w
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/ -x -q -m gpu --timeout 300 --timeout-method thread -rf > $O/gpu_tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -3 $O/gpu_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/sweep_batch.py --batches 64,128,256 --steps 60 > $O/sweep_10M.jsonl 2> $O/sweep_10M.err
rc=$?; echo "sweep 10M rc=$rc"; cat $O/sweep_10M.jsonl; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/sweep_batch.py --rows 1000000 --dim 768 --batches 64,128,256 --steps 100 > $O/sweep_c2.jsonl 2> $O/sweep_c2.err
rc=$?; echo "sweep c2 rc=$rc"; cat $O/sweep_c2.jsonl; [ $rc -ne 0 ] && exit $rc
for B in 128 256; do
  timeout -k 10 300 python -u bench.py --batch $B --steps 100 --warmup 10 > $O/bench_b$B.json 2> $O/bench_b$B.err
  rc=$?; echo "bench b$B rc=$rc"; tail -c 600 $O/bench_b$B.json; [ $rc -ne 0 ] && exit $rc
done
cd /tmp
R=$GRAFT_REPO_ROOT
for B in 128 256; do
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -T -d $R/$O/kt_b$B -o run --output-format csv -- python3 $R/bench.py --batch $B --steps 20 --warmup 5 --no-cpu > $R/$O/prof_kt_b$B.log 2>&1
  rc=$?; echo "kernel-trace b$B rc=$rc"; [ $rc -ne 0 ] && exit $rc
  timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_filter_wide|k_scan" -T -d $R/$O/fetch_b$B -o run --output-format csv -- python3 $R/bench.py --batch $B --steps 10 --warmup 2 --no-cpu > $R/$O/prof_fetch_b$B.log 2>&1
  rc=$?; echo "fetch b$B rc=$rc"; [ $rc -ne 0 ] && exit $rc
  timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "k_filter_wide|k_scan" -T -d $R/$O/write_b$B -o run --output-format csv -- python3 $R/bench.py --batch $B --steps 10 --warmup 2 --no-cpu > $R/$O/prof_write_b$B.log 2>&1
  rc=$?; echo "write b$B rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0

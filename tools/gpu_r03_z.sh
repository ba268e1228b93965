# round 3: k = 100 refresh-interval A/B (10M, B = 64); rocprofv3 of the final 128-query FILTER at B = 128 / 256
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r03z
mkdir -p $O
for cfg in "HIPRAG_REFRESH=4" "HIPRAG_REFRESH=8" "HIPRAG_REFRESH=16" "HIPRAG_REFRESH=4"; do
  env $cfg timeout -k 10 300 python -u bench.py --k 100 --steps 100 --warmup 10 --no-cpu > $O/k100.json 2> $O/k100.err || { echo "$cfg failed"; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/k100.json').read().strip().splitlines()[-1]); print('k=100 $cfg', d['ms_per_step'], d['roofline']['avg_launch_ms'])" | tee -a $O/k100_refresh_ab.log
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
  timeout -k 10 300 python3 $R/bench.py --batch $B --steps 100 --warmup 10 > $R/$O/bench_b$B.json 2> $R/$O/bench_b$B.err
  rc=$?; echo "bench b$B rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0

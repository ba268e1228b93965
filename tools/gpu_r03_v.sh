# round 3: B = 128 / 256 on the 128-query FILTER: all CUs vs n_cu - 32 for the pipelined scan, then rocprofv3 of
# the exact bench command at B = 128 (kernel trace + stats, then FETCH_SIZE / WRITE_SIZE passes)
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r03v
mkdir -p $O
HIPRAG_TAIL_CUS=0 timeout -k 10 300 python -u tools/sweep_batch.py --batches 128,256 --steps 60 > $O/sweep_tail0.jsonl 2> $O/sweep_tail0.err
echo "sweep tail0 rc=$?"; cat $O/sweep_tail0.jsonl
timeout -k 10 300 python -u bench.py --batch 128 --steps 50 --warmup 5 --no-cpu > $O/bench_b128.json 2> $O/bench_b128.err
rc=$?; echo "bench b128 rc=$rc"; tail -1 $O/bench_b128.json; [ $rc -ne 0 ] && exit $rc
cd /tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 600 rocprofv3 --kernel-trace --stats -T -d $R/$O/kt -o run --output-format csv -- python3 $R/bench.py --batch 128 --steps 20 --warmup 5 --no-cpu > $R/$O/prof_kt.log 2>&1
rc=$?; echo "kernel-trace rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_filter_wide|k_scan" -T -d $R/$O/pmc_fetch -o run --output-format csv -- python3 $R/bench.py --batch 128 --steps 10 --warmup 2 --no-cpu > $R/$O/prof_fetch.log 2>&1
rc=$?; echo "pmc fetch rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "k_filter_wide|k_scan" -T -d $R/$O/pmc_write -o run --output-format csv -- python3 $R/bench.py --batch 128 --steps 10 --warmup 2 --no-cpu > $R/$O/prof_write.log 2>&1
echo "pmc write rc=$?"

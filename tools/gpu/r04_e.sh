# r04 e: triple-buffered 128-query FILTER (parity + A/B against the previous kernel in ab/libhiprag_oldwide.so),
# persistent FILTER timeline at 1.25M rows, then PMC passes on k_filter_wide8 (B=128) and k_scan_filter (B=64)
set -u
O=gpurun_out/r04e; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_index.py -k "wide or tiles" tests/test_gpu_persist.py > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "passed|failed|error" $O/tests.log | tail -3; [ $rc -ne 0 ] && exit $rc
run() {  # tag, env prefix, args
  tag=$1; shift
  timeout -k 10 240 "$@" --no-cpu --no-embed --steps 30 --warmup 5 > $O/$tag.json 2> $O/$tag.err; rc=$?
  echo "$tag rc=$rc"; [ $rc -ne 0 ] && { tail -5 $O/$tag.err; exit $rc; }
  python3 -c "import json,sys;d=json.load(open('$O/$tag.json'));r=d['roofline'];print(d['value'],d['ms_per_step'],r['avg_launch_ms'],r['frac'],d.get('persist_timeline'))"
}
for rep in 1 2; do
  run b128_new_$rep python3 bench.py --batch 128
  HIPRAG_LIB_OVERRIDE=ab/libhiprag_oldwide.so run b128_old_$rep python3 bench.py --batch 128
done
run b256_new python3 bench.py --batch 256
HIPRAG_LIB_OVERRIDE=ab/libhiprag_oldwide.so run b256_old python3 bench.py --batch 256
run shard_p1 python3 bench.py --rows 1250000 --persist 1
run shard_p0 python3 bench.py --rows 1250000 --persist 0
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS"
P2="SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INST_LEVEL_VMEM SQ_INSTS_MFMA SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_ANY"
P3="TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_LFIFO_STALL_CYCLES_sum TCP_RFIFO_STALL_CYCLES_sum"
P4="FETCH_SIZE"
for B in 128 64; do
  i=0
  for P in "$P1" "$P2" "$P3" "$P4"; do
    i=$((i+1))
    timeout -s KILL 240 rocprofv3 --pmc $P --kernel-include-regex "k_filter_wide8|k_scan_filter" -T -d $O/b${B}_p$i -o run --output-format csv -- python3 bench.py --batch $B --steps 10 --warmup 2 --no-cpu --no-embed > $O/b${B}_p$i.log 2>&1; rc=$?
    echo "B=$B pass $i rc=$rc"; [ $rc -ne 0 ] && { tail -5 $O/b${B}_p$i.log; exit $rc; }
  done
done

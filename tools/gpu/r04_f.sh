# r04 f: 128-query FILTER diagnostics (barrier-free / staging-free builds, wrong results, timing only) against the
# product kernel; persistent FILTER vs per-batch launches over shard sizes; PMC passes on the product k_filter_wide8
set -u
O=gpurun_out/r04f; mkdir -p $O
export TMPDIR=/tmp
run() {  # tag, command...
  tag=$1; shift
  timeout -k 10 240 "$@" --no-cpu --no-embed --steps 30 --warmup 5 > $O/$tag.json 2> $O/$tag.err; rc=$?
  echo "$tag rc=$rc"; [ $rc -ne 0 ] && { tail -5 $O/$tag.err; exit $rc; }
  python3 -c "import json,sys;d=json.load(open('$O/$tag.json'));r=d['roofline'];print(d['value'],d['ms_per_step'],r['avg_launch_ms'],r['frac'],d.get('persist_timeline'))"
}
for rep in 1 2; do
  run b128_prod_$rep python3 bench.py --batch 128
  HIPRAG_LIB_OVERRIDE=ab/libhiprag_wide_nobarrier.so run b128_nobarrier_$rep python3 bench.py --batch 128
  HIPRAG_LIB_OVERRIDE=ab/libhiprag_wide_nostage.so run b128_nostage_$rep python3 bench.py --batch 128
done
for rows in 625000 1250000 2500000 5000000; do
  run r${rows}_p0 python3 bench.py --rows $rows --persist 0
  run r${rows}_p1 python3 bench.py --rows $rows --persist 1
done
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS"
P2="SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INST_LEVEL_VMEM SQ_INSTS_MFMA SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_ANY"
P3="TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_LFIFO_STALL_CYCLES_sum TCP_RFIFO_STALL_CYCLES_sum"
P4="FETCH_SIZE"
i=0
for P in "$P1" "$P2" "$P3" "$P4"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $P --kernel-include-regex "k_filter_wide8" -T -d $O/b128_p$i -o run --output-format csv -- python3 bench.py --batch 128 --steps 10 --warmup 2 --no-cpu --no-embed > $O/b128_p$i.log 2>&1; rc=$?
  echo "B=128 pass $i rc=$rc"; if [ $rc -ne 0 ]; then tail -5 $O/b128_p$i.log; exit $rc; fi
done
echo done

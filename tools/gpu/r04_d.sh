# r04 d: PMC passes on the 128-query FILTER (k_filter_wide8, bench --batch 128) and, for comparison, the 64-query
# k_scan_filter (bench default): stall / LDS / MFMA / TCP counters, one rocprofv3 pass per counter group
set -u
O=gpurun_out/r04d; mkdir -p $O
export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS"
P2="SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INST_LEVEL_VMEM SQ_INSTS_MFMA SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_ANY"
P3="TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_LFIFO_STALL_CYCLES_sum TCP_RFIFO_STALL_CYCLES_sum"
P4="FETCH_SIZE"
for B in 128 64; do
  i=0
  for P in "$P1" "$P2" "$P3" "$P4"; do
    i=$((i+1))
    timeout -s KILL 240 rocprofv3 --pmc $P --kernel-include-regex "k_filter_wide8|k_scan_filter" -T -d $O/b${B}_p$i -o run --output-format csv -- python3 bench.py --batch $B --steps 10 --warmup 2 --no-cpu > $O/b${B}_p$i.log 2>&1; rc=$?
    echo "B=$B pass $i rc=$rc"; [ $rc -ne 0 ] && { tail -5 $O/b${B}_p$i.log; exit $rc; }
  done
done

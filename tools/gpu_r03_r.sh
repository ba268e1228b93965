# round 3: SQ counters of the 128-query FILTER (real kernel, 10M x 1024, B = 128) vs its timing prototype
set -o pipefail
cd /tmp && export TMPDIR=/tmp PYTHONUNBUFFERED=1
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r03u
mkdir -p $O
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS"
P2="SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAIT_INST_LDS"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --kernel-include-regex k_filter_wide -d $O/real$i -o pmc --output-format csv -- python3 $R/tools/diag_wide.py --reps 5 > $O/real$i.log 2>&1 || { echo "real pass $i failed"; tail -5 $O/real$i.log; exit 1; }
  timeout -s KILL 60 rocprofv3 --pmc $P -d $O/proto$i -o pmc --output-format csv -- $R/tools/q128_proto 20.48 3 > $O/proto$i.log 2>&1 || { echo "proto pass $i failed"; tail -5 $O/proto$i.log; exit 1; }
done
find $O -name "*counter_collection*"

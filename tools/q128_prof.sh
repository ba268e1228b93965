set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/q128pmc
mkdir -p $O
for v in 0 4; do
timeout -s KILL 60 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_BUSY_CYCLES -d $O/v$v -o pmc -- $R/tools/q128_proto 20.48 $v > $O/v$v.log 2>&1 || exit 1
timeout -s KILL 60 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_COEXEC_CYCLES GRBM_GUI_ACTIVE -d $O/w$v -o pmc -- $R/tools/q128_proto 20.48 $v > $O/w$v.log 2>&1 || echo "second pass failed"
done
ls -R $O | head -30

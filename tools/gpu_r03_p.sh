# round 3: 128-query FILTER diagnostics (candidates, FILTER time) vs query groups and A/B builds
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r03p
mkdir -p $O
L=youtu-rag_amd/hiprag
for cfg in "HIPRAG_WIDE_FILTER=1" "HIPRAG_LIB_OVERRIDE=$L/libhiprag_noapp.so"; do
  env $cfg timeout -k 10 200 python -u tools/diag_wide.py --reps 20 >> $O/diag.jsonl 2>> $O/diag.err || { echo "$cfg failed"; exit 1; }
  tail -1 $O/diag.jsonl
done

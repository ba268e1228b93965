# round 3: refreshes of the 128-query FILTER staggered over the workgroups (HR_WIDE_STAGGER) vs all at once
# (libhiprag_nostagger.so), refresh every 1 / 2 / 4 rounds: FILTER time and candidates at 10M x 1024, B = 128
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r03ag
mkdir -p $O
L=youtu-rag_amd/hiprag
timeout -k 10 600 python -u -m pytest tests/test_gpu_index.py -x -q --timeout 300 --timeout-method thread -k "wide" > $O/wide_tests.log 2>&1
rc=$?; echo "wide tests rc=$rc"; tail -2 $O/wide_tests.log; [ $rc -ne 0 ] && exit $rc
for k in 10 50; do
  for rt in 1 2 4; do
    for lib in "" "$L/libhiprag_nostagger.so"; do
      HIPRAG_REFRESH=$rt HIPRAG_LIB_OVERRIDE=$lib timeout -k 10 200 python -u tools/diag_wide.py --reps 10 --k $k >> $O/diag.jsonl 2>> $O/diag.err || { echo "diag failed"; exit 1; }
      echo "rt=$rt $(tail -1 $O/diag.jsonl | cut -c1-330)"
    done
  done
done
exit 0

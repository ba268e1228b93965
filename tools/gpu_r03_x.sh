# round 3: 128-query FILTER -- spare CUs for an early SAMPLE (HIPRAG_WIDE_TAIL_CUS) and the SAMPLE size, B = 128
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r03x
mkdir -p $O
for rows in 10000000 1250000; do
for cfg in "HIPRAG_WIDE_TAIL_CUS=0" "HIPRAG_WIDE_TAIL_CUS=8" "HIPRAG_WIDE_TAIL_CUS=16" "HIPRAG_SAMPLE_MIN=1024" "HIPRAG_SAMPLE_MIN=512"; do
  env $cfg timeout -k 10 200 python -u tools/sweep_batch.py --rows $rows --batches 128 --steps 100 > $O/s.jsonl 2> $O/s.err || { echo "$cfg failed"; exit 1; }
  echo "$rows $cfg: $(tail -1 $O/s.jsonl)" | tee -a $O/ab.log
done
done
exit 0

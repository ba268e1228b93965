# round 3: row parts in the 128-query FILTER, pipelined batch sweeps (the bench's path) at 10M x 1024: bf16 k = 20 / 50,
# fp32 k = 20 / 50 / 100, parts allowed (99) vs query groups (1)
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r03af
mkdir -p $O
for k in 20 50; do
  for wp in 99 1; do
    HIPRAG_WIDE_PARTS=$wp timeout -k 10 300 python -u tools/sweep_batch.py --batches 128,256 --k $k --steps 40 > $O/s.jsonl 2>> $O/sweep.err || { echo "bf16 k=$k wp=$wp failed"; exit 1; }
    sed "s/^/{\"parts_max\": $wp, \"dtype\": \"bf16\", \"row\": /; s/$/}/" $O/s.jsonl >> $O/sweep.jsonl; cat $O/s.jsonl
  done
done
for k in 20 50 100; do
  for wp in 99 1; do
    HIPRAG_WIDE_PARTS=$wp timeout -k 10 300 python -u tools/sweep_batch.py --dtype f32 --batches 128 --k $k --steps 30 > $O/s.jsonl 2>> $O/sweep.err || { echo "f32 k=$k wp=$wp failed"; exit 1; }
    sed "s/^/{\"parts_max\": $wp, \"dtype\": \"f32\", \"row\": /; s/$/}/" $O/s.jsonl >> $O/sweep.jsonl; cat $O/s.jsonl
  done
done
exit 0

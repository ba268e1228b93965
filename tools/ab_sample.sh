# A/B: SAMPLE pass with default-policy loads (served from the Infinity Cache after the first batch) vs nt
set -e
for rep in 1 2; do
  for v in 0 1; do
    HIPRAG_SAMPLE_NT=$v timeout -k 10 120 python -u bench.py --rows 1250000 --steps 300 --warmup 10 --no-cpu > gpurun_out/abs_1.25M_nt${v}_$rep.json 2>/dev/null
    HIPRAG_SAMPLE_NT=$v timeout -k 10 120 python -u bench.py --rows 2500000 --steps 200 --warmup 10 --no-cpu > gpurun_out/abs_2.5M_nt${v}_$rep.json 2>/dev/null
  done
done
HIPRAG_SAMPLE_NT=0 timeout -k 10 200 python -u bench.py --steps 100 --warmup 5 --no-cpu > gpurun_out/abs_10M_nt0.json 2>/dev/null
HIPRAG_SAMPLE_NT=1 timeout -k 10 200 python -u bench.py --steps 100 --warmup 5 --no-cpu > gpurun_out/abs_10M_nt1.json 2>/dev/null

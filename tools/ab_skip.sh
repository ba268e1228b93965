# A/B: sampled tiles scored once (SAMPLE keeps its buckets, the FILTER skips its tiles) vs read twice
set -e
mkdir -p gpurun_out
for rep in 1 2; do
  for v in 0 1; do
    HIPRAG_SAMPLE_SKIP=$v timeout -k 10 120 python -u bench.py --rows 1250000 --steps 300 --warmup 10 --no-cpu > gpurun_out/abk_1.25M_s${v}_$rep.json 2>/dev/null
    HIPRAG_SAMPLE_SKIP=$v timeout -k 10 120 python -u bench.py --rows 2500000 --steps 200 --warmup 10 --no-cpu > gpurun_out/abk_2.5M_s${v}_$rep.json 2>/dev/null
  done
done
for v in 0 1; do
  HIPRAG_SAMPLE_SKIP=$v timeout -k 10 200 python -u bench.py --steps 100 --warmup 5 --no-cpu > gpurun_out/abk_10M_s${v}.json 2>/dev/null
done
for f in gpurun_out/abk_*.json; do echo "$f $(python3 -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['frac'])")"; done

# A/B: sample size of small shards (HIPRAG_SAMPLE_FRAC: 8 = at most 1/8 of the shard, 0 = fixed 2048 tiles)
set -e
timeout -k 10 300 python -u -m pytest tests/test_gpu_index.py -x -q --timeout 120 --timeout-method thread > gpurun_out/sfrac_tests.log 2>&1
for rep in 1 2; do
  for v in 8 0; do
    HIPRAG_SAMPLE_FRAC=$v timeout -k 10 120 python -u bench.py --rows 100000 --steps 500 --warmup 20 --no-cpu > gpurun_out/absf_100k_${v}_$rep.json 2>/dev/null
    HIPRAG_SAMPLE_FRAC=$v timeout -k 10 120 python -u bench.py --rows 300000 --steps 400 --warmup 20 --no-cpu > gpurun_out/absf_300k_${v}_$rep.json 2>/dev/null
    HIPRAG_SAMPLE_FRAC=$v timeout -k 10 120 python -u bench.py --rows 1000000 --dim 768 --steps 300 --warmup 10 --no-cpu > gpurun_out/absf_c2_${v}_$rep.json 2>/dev/null
  done
done

# A/B: swapped-pair tile order for odd query groups (HIPRAG_GROUP_SWAP) at B = 128 / 256, 10M rows
set -e
timeout -k 10 300 python -u -m pytest tests/test_gpu_index.py -x -q -k "query_groups" --timeout 120 --timeout-method thread > gpurun_out/swap_tests.log 2>&1
for rep in 1 2; do
  for v in 1 0; do
    HIPRAG_GROUP_SWAP=$v timeout -k 10 300 python -u tools/sweep_batch.py --batches 128,256 --steps 30 > gpurun_out/abswap_${v}_$rep.jsonl 2>/dev/null
  done
done

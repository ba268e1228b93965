# A/B of the query-group scan variants at 10M x 1024 bf16 (B = 128, 256): 4 waves/CU with a 64- or
# 32-deep ring vs 8 waves/CU with a 16-deep ring.
set -e
timeout -k 10 200 python -u -m pytest tests/test_gpu_index.py -x -q -k "query_groups" --timeout 150 --timeout-method thread > gpurun_out/abg_tests.log 2>&1
for v in "HIPRAG_GROUP_RING=64" "HIPRAG_GROUP_RING=32" "HIPRAG_GROUP_TPB=512"; do
  env $v timeout -k 10 200 python -u tools/sweep_batch.py --batches 128,256 --steps 30 > gpurun_out/abg_$(echo $v | tr '=' '_').jsonl 2>/dev/null
done

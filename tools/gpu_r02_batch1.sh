# one GPU call: query-group and IVF parity, the group-scan A/B, the streaming ceiling, the IVF bench
set -e
timeout -k 10 300 python -u -m pytest tests/test_gpu_index.py tests/test_gpu_ivf.py -x -q -k "query_groups or ivf" --timeout 150 --timeout-method thread > gpurun_out/b1_tests.log 2>&1
for v in "HIPRAG_GROUP_RING=64" "HIPRAG_GROUP_RING=32" "HIPRAG_GROUP_TPB=512"; do
  env $v timeout -k 10 200 python -u tools/sweep_batch.py --batches 128,256 --steps 30 > gpurun_out/abg_$(echo $v | tr '=' '_').jsonl 2>/dev/null
done
timeout -k 10 120 ./tools/stream_ceiling 20.48 > gpurun_out/stream_ceiling2.jsonl 2>&1
timeout -k 10 60 ./tools/stream_ceiling 2.56 >> gpurun_out/stream_ceiling2.jsonl 2>&1
timeout -k 10 300 python3 tools/bench_ivf.py > gpurun_out/ivf_r02b.jsonl 2> gpurun_out/ivf_r02b.err

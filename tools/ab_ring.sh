# A/B: corpus ring kept in issue order (sched barriers, scalar live/mask, default) vs the compiler's
# schedule (libhiprag_ab.so built with -DHR_RING_SCHED=0); quick parity first
set -e
HIPRAG_LIB_OVERRIDE=$PWD/youtu-rag_amd/hiprag/libhiprag_ab.so timeout -k 10 300 python -u -m pytest tests/test_gpu_index.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ring_tests.log 2>&1
for rep in 1 2; do
  for lib in youtu-rag_amd/hiprag/libhiprag.so youtu-rag_amd/hiprag/libhiprag_ab.so; do
    tag=$(basename $lib .so)_$rep
    HIPRAG_LIB_OVERRIDE=$PWD/$lib timeout -k 10 120 python -u bench.py --rows 1250000 --steps 300 --warmup 10 --no-cpu > gpurun_out/abring_1.25M_$tag.json 2>/dev/null
    HIPRAG_LIB_OVERRIDE=$PWD/$lib timeout -k 10 200 python -u bench.py --steps 100 --warmup 5 --no-cpu > gpurun_out/abring_10M_$tag.json 2>/dev/null
  done
done
for lib in youtu-rag_amd/hiprag/libhiprag.so youtu-rag_amd/hiprag/libhiprag_ab.so; do
  HIPRAG_LIB_OVERRIDE=$PWD/$lib timeout -k 10 300 python -u tools/sweep_batch.py --batches 128,256 --steps 30 > gpurun_out/abring_groups_$(basename $lib .so).jsonl 2>/dev/null
done

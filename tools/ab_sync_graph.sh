#!/bin/bash
# A/B of the synchronous search's HIP graph replay under the store's async micro-batcher (batch sizes
# vary from launch to launch, so the (B, k) shapes churn): 100k rows, 1..256 clients, graphs on / off.
set -e
for g in 1 0; do
    echo "# HIPRAG_SYNC_GRAPH=$g"
    HIPRAG_SYNC_GRAPH=$g timeout -k 10 250 python -u tools/bench_async.py --rows 100000 --clients 1,16,64,256,1024 \
        --max-batch 64 --seconds 2 --gc-freeze 1
done

#!/bin/bash
# A/B: static scan units as contiguous per-wave ranges (HIPRAG_STRIDED=0) vs dealt round-robin (1),
# alternated twice: 10M rows B = 64 / 128 (sweep) and the 1.25M-row shard (bench.py).
set -e
for rep in 1 2; do
    for s in 0 1; do
        echo "# HIPRAG_STRIDED=$s rep $rep"
        HIPRAG_STRIDED=$s timeout -k 10 200 python -u tools/sweep_batch.py --batches 64,128 --steps 40
        HIPRAG_STRIDED=$s timeout -k 10 200 python -u bench.py --rows 1250000 --steps 200 --warmup 20 2>/dev/null
    done
done

#!/bin/bash
# A/B of the wide FILTER (k_scan_wide) at 10M x 1024 bf16: ring depth and what bounds a stage
# (HIPRAG_WIDE_DEBUG=1 drops the MFMAs, 2 the LDS reads too -- timing only, results wrong).
set -e
for cfg in "HIPRAG_WIDE=0" "HIPRAG_WIDE=1" "HIPRAG_WIDE_RING=8" "HIPRAG_WIDE_DEBUG=1" "HIPRAG_WIDE_DEBUG=2"; do
    echo "# $cfg"
    env $cfg timeout -k 10 200 python -u tools/sweep_batch.py --batches 128,256 --steps 30
done

#!/usr/bin/env python3
"""Diagnostics of the 128-query FILTER (hr_wide.hip) at a BASELINE shard size: synchronous searches of B planted
queries, printing the FILTER's HIP-event time, candidates appended (total / max per query) and guard failures.
Run it once with HIPRAG_WIDE_FILTER=0 (query groups) and once without to compare; HIPRAG_LIB_OVERRIDE selects an
A/B build of the library.
Usage: python tools/diag_wide.py [--rows N] [--dim D] [--batch B] [--k K] [--reps R]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "youtu-rag_amd")]

import numpy as np  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=10_000_000)
    ap.add_argument("--dim", type=int, default=1024)
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--dtype", default="bf16")
    args = ap.parse_args()
    import torch

    from hiprag import _native, synth

    idx = _native.NativeIndex(args.dim, args.dtype, "cosine")
    idx.reserve(args.rows)
    idx.add_synthetic(0, 0, args.rows)
    torch.cuda.synchronize()
    q, _ = synth.planted_queries(0, args.rows, args.dim, args.batch, qseed=1000)
    idx.search(q, args.k)  # warm
    idx.set_scan_timing(1)
    idx.take_scan_times()
    t0 = time.perf_counter()
    cands = []
    for i in range(args.reps):
        q, _ = synth.planted_queries(0, args.rows, args.dim, args.batch, qseed=1001 + i)
        idx.search(q, args.k)
        cands.append(idx.last_candidates())
    wall = (time.perf_counter() - t0) / args.reps
    sample_ms, filter_ms = idx.take_scan_times()
    st = idx.stats()
    print(json.dumps({"rows": args.rows, "dim": args.dim, "B": args.batch, "k": args.k,
                      "wide": os.environ.get("HIPRAG_WIDE_FILTER", "1"), "lib": os.environ.get("HIPRAG_LIB_OVERRIDE", ""),
                      "filter_ms": round(float(np.mean(filter_ms)), 4), "sample_ms": round(float(np.mean(sample_ms)), 4),
                      "wall_ms_per_search": round(1000 * wall, 3),
                      "cands_total_mean": float(np.mean([c[0] for c in cands])),
                      "cands_per_query_mean": float(np.mean([c[0] for c in cands])) / args.batch,
                      "cands_max_per_query": int(max(c[1] for c in cands)),
                      "guard_failures": st.get("guard_failures"), "passes": st.get("passes")}), flush=True)


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Batch-size sweep (B in {1, 16, 64, 256}) at 10M x 1024 bf16, one GPU.

For each B: throughput of the pipelined path the bench times (ShardedSearch, batches in flight,
queries resident in HBM) -> QPS and ms per batch, the FILTER scan's average launch time from HIP
events (-> scan GB/s and fraction of 8 TB/s), scan passes per batch (hr_index_stats), and the
synchronous single-batch latency (submit + finalize of one batch at a time).  One JSON line per B.
Usage: python tools/sweep_batch.py [--rows N] [--dim D] [--batches 1,16,64,128,256] [--steps 60]
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
    ap.add_argument("--batches", default="1,16,64,128,256")
    ap.add_argument("--steps", type=int, default=60)
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--dtype", default="bf16")
    args = ap.parse_args()
    import torch

    from hiprag import _native, synth
    from hiprag.dist import ShardedSearch

    dev = torch.device("cuda", 0)
    idx = _native.NativeIndex(args.dim, args.dtype, "cosine")
    idx.reserve(args.rows)
    idx.add_synthetic(0, 0, args.rows)
    esz = 4 if args.dtype == "f32" else 2
    alg = args.rows * args.dim * esz
    for B in [int(x) for x in args.batches.split(",")]:
        nb = args.steps + 5
        q = torch.from_numpy(np.stack([synth.planted_queries(0, args.rows, args.dim, B, qseed=7000 + i)[0]
                                       for i in range(nb)])).to(dev)
        ready = torch.cuda.Event()
        ready.record()
        ss = ShardedSearch(idx, 0, max_batch=B, device=dev, max_k=max(16, args.k))
        s = torch.empty((nb, B, args.k), dtype=torch.float32, device=dev)
        r = torch.empty((nb, B, args.k), dtype=torch.int64, device=dev)
        for i in range(5):
            ss.submit(q[i], args.k, s_out=s[i], r_out=r[i], q_ready=ready)
        ss.finalize_all()
        torch.cuda.synchronize()
        idx.take_scan_times()
        idx.set_scan_timing(4)
        p0 = idx.stats()["main_passes"]
        t0 = time.perf_counter()
        for i in range(5, nb):
            ss.submit(q[i], args.k, s_out=s[i], r_out=r[i], q_ready=ready)
        ss.finalize_all()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        passes = (idx.stats()["main_passes"] - p0) / args.steps
        _, filt = idx.take_scan_times()
        idx.set_scan_timing(0)
        lat = []
        for i in range(5, min(nb, 25)):
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            ss.search(q[i], args.k, s_out=s[i], r_out=r[i])
            torch.cuda.synchronize()
            lat.append(1000 * (time.perf_counter() - t1))
        scan_ms = float(np.mean(filt)) if len(filt) else float("nan")
        print(json.dumps({"rows": args.rows, "dim": args.dim, "B": B, "k": args.k,
                          "qps": round(args.steps * B / dt, 1), "ms_per_batch": round(1000 * dt / args.steps, 4),
                          "scan_passes_per_batch": passes, "filter_ms": round(scan_ms, 4),
                          "scan_GBps": round(alg / (scan_ms * 1e-3) / 1e9, 1),
                          "frac_of_8TBps": round(alg / (scan_ms * 1e-3) / 8e12, 4),
                          "sync_latency_ms_p50": round(float(np.median(lat)), 3)}), flush=True)
        del ss


if __name__ == "__main__":
    main()

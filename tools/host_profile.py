#!/usr/bin/env python3
"""Host-side cost of one pipelined search step (ShardedSearch.submit/finalize) on a small collection,
where the GPU work per step is short and the host bounds the step: cProfile of N steps, top entries by
own time, plus the wall time per step.  Usage: python tools/host_profile.py [--rows 100000 --steps 500]"""
from __future__ import annotations

import argparse
import cProfile
import os
import pstats
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "youtu-rag_amd"), REPO]


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--rows", type=int, default=100_000)
    p.add_argument("--steps", type=int, default=500)
    args = p.parse_args()
    import numpy as np
    import torch

    from hiprag import _native, synth
    from hiprag.dist import ShardedSearch

    dev = torch.device("cuda", 0)
    D, B, K = 1024, 64, 10
    idx = _native.NativeIndex(D, "bf16", "cosine")
    idx.reserve(args.rows)
    idx.add_synthetic(0, 0, args.rows)
    q = torch.from_numpy(np.stack([synth.planted_queries(0, args.rows, D, B, qseed=i)[0] for i in range(8)])).to(dev)
    ready = torch.cuda.Event()
    ready.record()
    ss = ShardedSearch(idx, 0, max_batch=B, device=dev)
    s_out = torch.empty((8, B, K), dtype=torch.float32, device=dev)
    r_out = torch.empty((8, B, K), dtype=torch.int64, device=dev)
    for i in range(50):
        ss.submit(q[i % 8], K, s_out=s_out[i % 8], r_out=r_out[i % 8], q_ready=ready)
    ss.finalize_all()
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    t0 = time.perf_counter()
    pr.enable()
    for i in range(args.steps):
        ss.submit(q[i % 8], K, s_out=s_out[i % 8], r_out=r_out[i % 8], q_ready=ready)
    ss.finalize_all()
    pr.disable()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / args.steps
    print(f"rows {args.rows}: {dt * 1e3:.4f} ms per step (profiled)")
    pstats.Stats(pr).sort_stats("tottime").print_stats(18)


if __name__ == "__main__":
    main()

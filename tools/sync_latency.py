#!/usr/bin/env python3
"""Latency of the synchronous host-query search (NativeIndex.search = hr_index_search: H2D, scan,
rescore, merge, guard check, D2H) for small batches on collections of several sizes -- the path the
store's micro-batcher takes for a lone caller.  Usage: python tools/sync_latency.py [--rows 100000,1000000]"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "youtu-rag_amd"), REPO]


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--rows", default="10000,100000,1000000")
    p.add_argument("--batches", default="1,16,64")
    p.add_argument("--calls", type=int, default=200)
    args = p.parse_args()
    import numpy as np

    from hiprag import _native, synth

    for n in (int(x) for x in args.rows.split(",")):
        idx = _native.NativeIndex(1024, "bf16", "cosine")
        idx.reserve(n)
        idx.add_synthetic(0, 0, n)
        for B in (int(x) for x in args.batches.split(",")):
            q, _ = synth.planted_queries(0, n, 1024, B, qseed=3)
            for _ in range(10):
                idx.search(q, 10)
            lat = []
            for _ in range(args.calls):
                t0 = time.perf_counter()
                idx.search(q, 10)
                lat.append(time.perf_counter() - t0)
            a = np.asarray(lat) * 1e3
            print(json.dumps({"rows": n, "B": B, "ms_p50": round(float(np.percentile(a, 50)), 4),
                              "ms_p99": round(float(np.percentile(a, 99)), 4)}), flush=True)
        idx.close()


if __name__ == "__main__":
    main()

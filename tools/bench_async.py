#!/usr/bin/env python3
"""The reference's call pattern through the drop-in store: many concurrent single-query
``await store.search(query_embedding=..., top_k=10)`` calls (VectorRetriever.retrieve,
base_retriever.py:58-63), coalesced by HipVectorStore's micro-batcher into batched launches.

Builds a HipVectorStore over n synthetic rows (10M x 1024 bf16 by default, 1000-chunk documents, as
tools/bench_filter.py STORE=1), then for each concurrency C runs C client coroutines that each issue
sequential searches with planted queries for a fixed wall time, and reports queries/s, latency
percentiles, the mean launch size and launches.  One JSON line per (max_batch, C).
Usage: python tools/bench_async.py [--rows 10000000 --clients 1,16,64,256,1024 --max-batch 64,256 --seconds 3]
"""
from __future__ import annotations

import argparse
import asyncio
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "youtu-rag_amd"), REPO]


def build_store(n: int, max_batch: int, idx=None, dtype: str = "bf16"):
    from hiprag import _native
    from hiprag.rag import HipVectorStore, VectorStoreConfig

    D = 1024
    if idx is None:
        idx = _native.NativeIndex(D, dtype, "cosine")
        idx.reserve(n)
        idx.add_synthetic(0, 0, n)
    cfg = VectorStoreConfig(backend="hip", collection_name="bench", persist_directory="/tmp/hiprag_bench_async",
                            index_params={"dtype": dtype, "persist": False, "max_batch": max_batch})
    st = HipVectorStore(cfg, index_factory=lambda d: idx)
    st._ensure_index(D)
    recs = []
    for r in range(n):
        d, i = divmod(r, 1000)
        recs.append({"id": f"doc{d}_chunk_{i}", "document_id": f"doc{d}", "content": "", "chunk_index": i,
                     "metadata": {"document_id": f"doc{d}", "chunk_index": i}})
        if len(recs) == 1_000_000:
            st._append_tables(recs, None)
            recs = []
    if recs:
        st._append_tables(recs, None)
    return st, idx


async def run_clients(st, queries, C: int, seconds: float, k: int):
    lat: list[float] = []
    stop = time.perf_counter() + seconds
    nq = len(queries)

    async def client(c):
        j = c
        while time.perf_counter() < stop:
            t0 = time.perf_counter()
            res = await st.search(query_embedding=queries[j % nq], top_k=k)
            lat.append(time.perf_counter() - t0)
            assert len(res) == k
            j += C

    launches0 = st._batcher.launches
    t0 = time.perf_counter()
    await asyncio.gather(*(client(c) for c in range(C)))
    wall = time.perf_counter() - t0
    return lat, wall, st._batcher.launches - launches0


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--rows", type=int, default=10_000_000)
    p.add_argument("--clients", default="1,16,64,256,1024")
    p.add_argument("--max-batch", default="64,256")
    p.add_argument("--depth", default="2", help="launches in flight (comma list: A/B)")
    p.add_argument("--gc-freeze", default="0", help="0/1 list: gc.freeze() after building the store (A/B)")
    p.add_argument("--seconds", type=float, default=3.0)
    p.add_argument("--k", type=int, default=10)
    p.add_argument("--dtype", default="bf16", help="stored rows: bf16, or f32 (the store's default, the reference's)")
    p.add_argument("--native-async", default="1", help="0/1 list: event-loop native launches (1) or worker threads (0)")
    p.add_argument("--torch", type=int, default=1,
                   help="import torch first: a serving process's heap (the in-process embedder), ~170k tracked objects "
                        "that every full collection walks unless the application froze them")
    p.add_argument("--profile", default="", help="write a cProfile summary of each measured run to PATH.<clients>_<mb>")
    args = p.parse_args()

    import gc

    gc_time = [0.0, 0.0, 0.0]  # seconds inside collections, per generation
    gc_t0 = [0.0]

    def on_gc(phase, info):
        if phase == "start":
            gc_t0[0] = time.perf_counter()
        else:
            gc_time[info["generation"]] += time.perf_counter() - gc_t0[0]

    gc.callbacks.append(on_gc)

    if args.torch:
        import torch  # noqa: F401

    import numpy as np

    from hiprag import synth

    q, _ = synth.planted_queries(0, args.rows, 1024, 2048, qseed=11)
    queries = [np.asarray(x, np.float32) for x in q]
    t0 = time.perf_counter()
    st, _ = build_store(args.rows, 64, dtype=args.dtype)
    print(f"# store of {args.rows} rows in {time.perf_counter() - t0:.1f}s", file=sys.stderr, flush=True)
    t0 = time.perf_counter()
    gc.collect()
    print(f"# full collection {1e3 * (time.perf_counter() - t0):.1f} ms over {len(gc.get_objects())} tracked objects",
          file=sys.stderr, flush=True)
    for fz in (int(x) for x in args.gc_freeze.split(",")):
        if fz:
            gc.collect()
            gc.freeze()
        for depth, mb, na in ((d, m, a) for d in (int(x) for x in args.depth.split(","))
                              for m in (int(x) for x in args.max_batch.split(","))
                              for a in (int(x) for x in args.native_async.split(","))):
            st._batcher.max_batch, st._batcher.depth, st.native_async = mb, depth, bool(na)
            asyncio.run(run_clients(st, queries, 64, 0.5, args.k))  # warm
            for C in (int(x) for x in args.clients.split(",")):
                gc0 = [s["collections"] for s in gc.get_stats()]
                gct0 = list(gc_time)
                nat0 = st._batcher.native_launches
                if args.profile:
                    import cProfile
                    import pstats

                    prof = cProfile.Profile()
                    prof.enable()
                lat, wall, launches = asyncio.run(run_clients(st, queries, C, args.seconds, args.k))
                if args.profile:
                    prof.disable()
                    with open(f"{args.profile}.{C}_{mb}", "w") as f:
                        pstats.Stats(prof, stream=f).sort_stats("tottime").print_stats(30)
                a = np.asarray(lat) * 1e3
                print(json.dumps({"rows": args.rows, "dtype": args.dtype, "max_batch": mb, "depth": depth, "gc_freeze": fz,
                                  "native_async": na, "native_launches": st._batcher.native_launches - nat0,
                                  "clients": C,
                                  "queries": len(lat), "qps": round(len(lat) / wall, 1),
                                  "latency_ms_p50": round(float(np.percentile(a, 50)), 3),
                                  "latency_ms_p99": round(float(np.percentile(a, 99)), 3),
                                  "launches": launches, "mean_launch_size": round(len(lat) / max(1, launches), 1),
                                  "gc_collections": sum(s["collections"] for s in gc.get_stats()) - sum(gc0),
                                  "gc_collections_per_gen": [s["collections"] - c for s, c in zip(gc.get_stats(), gc0)],
                                  "gc_ms_per_gen": [round(1e3 * (t - t0), 1) for t, t0 in zip(gc_time, gct0)],
                                  "profiled": bool(args.profile)}),
                      flush=True)


if __name__ == "__main__":
    main()

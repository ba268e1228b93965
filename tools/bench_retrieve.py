#!/usr/bin/env python3
"""The reference's query path under concurrent callers: C client coroutines each call
``VectorRetriever.retrieve(query)`` in a loop (base_retriever.py:53-59: embed_query, then store.search with
``query_embedding=``), against a HipVectorStore of N synthetic rows and the in-process bge-large-shaped embedder
(random init, bf16).  One JSON line per (mode, clients): throughput, latency, forwards and launches.  Modes: ``fused`` -- the retriever's
cohorts (one forward whose output goes straight into one device-query store search, retriever._FusedRetrieve);
``coalesce`` -- the reference's two awaits with the embedder's query coalescer and the store's micro-batcher;
``percall`` -- one forward per call on the event loop.
Usage: python tools/bench_retrieve.py [--rows 10000000 --clients 64,256 --modes fused,coalesce --seconds 4]"""
from __future__ import annotations

import argparse
import asyncio
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "youtu-rag_amd"), REPO, os.path.join(REPO, "tools")]


def queries(n: int, seed: int = 5) -> list[str]:
    import random

    r = random.Random(seed)
    words = [f"term{i}" for i in range(5000)]
    return [" ".join(r.choice(words) for _ in range(r.randint(6, 20))) + "?" for _ in range(n)]


async def clients(ret, qs, C: int, seconds: float, k: int):
    lat: list[float] = []
    stop = time.perf_counter() + seconds

    async def client(c):
        j = c
        while time.perf_counter() < stop:
            t0 = time.perf_counter()
            res = await ret.retrieve(qs[j % len(qs)], top_k=k)
            lat.append(time.perf_counter() - t0)
            assert len(res) == k
            j += C

    t0 = time.perf_counter()
    await asyncio.gather(*(client(c) for c in range(C)))
    return lat, time.perf_counter() - t0


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--rows", type=int, default=10_000_000)
    p.add_argument("--clients", default="64,256")
    p.add_argument("--modes", default="fused,coalesce")
    p.add_argument("--seconds", type=float, default=4.0)
    p.add_argument("--k", type=int, default=10)
    p.add_argument("--max-batch", type=int, default=64, help="store search batches (and the embedder's batch_size)")
    p.add_argument("--embed-batch", default="64", help="comma list: queries per coalesced forward (A/B)")
    p.add_argument("--profile", default="", help="write a cProfile summary (event-loop thread) to PATH.<clients>")
    # application choices, not library policy (A/B of the cycle collector's share): the store's opt-in untracked results
    # (index_params.untracked_results), or the application's own gc.freeze() after its setup
    p.add_argument("--untracked", action="store_true")
    p.add_argument("--gc-freeze", action="store_true")
    a = p.parse_args()

    import numpy as np
    import torch  # noqa: F401

    from bench_async import build_store
    from hiprag.rag import RetrieverConfig, VectorRetriever
    from hiprag.rag.rocm_embedder import TorchRocmEmbedder, _QueryCoalescer

    t0 = time.perf_counter()
    st, _ = build_store(a.rows, a.max_batch)
    emb = TorchRocmEmbedder(preset="bge-large", dtype="bfloat16", batch_size=a.max_batch, max_length=512,
                            tuned_gemms=True)
    ret = VectorRetriever(st, emb, RetrieverConfig(top_k=a.k, similarity_threshold=0.0))
    qs = queries(4096)
    emb.encode_queries(qs[:a.max_batch])  # graph capture of the common shapes
    st.untracked_results = bool(a.untracked)
    if a.gc_freeze:
        import gc

        gc.collect()
        gc.freeze()
    print(f"# store of {a.rows} rows + embedder in {time.perf_counter() - t0:.1f}s", file=sys.stderr, flush=True)
    # the worker's time per forward, split: host tokenise + pack + launch, the device wait, the host lists
    wt = {"launch": 0.0, "wait": 0.0, "lists": 0.0, "n": 0}

    def timed_lists(qs_):
        t1 = time.perf_counter()
        x = emb.encode_queries(list(qs_))
        t2 = time.perf_counter()
        torch.cuda.synchronize()
        t3 = time.perf_counter()
        out = x.cpu().numpy().tolist()
        wt["launch"] += t2 - t1
        wt["wait"] += t3 - t2
        wt["lists"] += time.perf_counter() - t3
        wt["n"] += 1
        return out

    emb._query_lists = timed_lists
    fused = ret._fused
    for mode, eb in ((m, e) for m in a.modes.split(",") for e in (int(x) for x in a.embed_batch.split(","))):
        co = mode != "percall"
        ret._fused = fused if mode == "fused" else None
        if fused is not None:
            fused.max_batch = eb
        emb._coalescer = _QueryCoalescer(emb, eb) if mode == "coalesce" else None
        asyncio.run(clients(ret, qs, 64, 1.0, a.k))  # warm: the graphs of the batch shapes this mode makes
        for C in (int(x) for x in a.clients.split(",")):
            l0 = st._batcher.launches
            f0 = emb._coalescer.forwards if emb._coalescer else 0
            c0 = fused.cohorts if fused is not None else 0
            if fused is not None:
                fused.timing = {k: 0 for k in fused.timing}
            for key in wt:
                wt[key] = 0
            if a.profile:
                import cProfile
                import pstats

                prof = cProfile.Profile()
                prof.enable()
            lat, wall = asyncio.run(clients(ret, qs, C, a.seconds, a.k))
            if a.profile:
                prof.disable()
                with open(f"{a.profile}.{mode}.{C}", "w") as f:
                    pstats.Stats(prof, stream=f).sort_stats("tottime").print_stats(30)
            n = max(1, wt["n"])
            ms = np.asarray(lat) * 1e3
            fw = (fused.cohorts - c0) if mode == "fused" else (emb._coalescer.forwards - f0) if co else len(lat)
            print(json.dumps({"rows": a.rows, "mode": mode, "embed_batch": eb if co else 1, "clients": C,
                              "queries": len(lat), "qps": round(len(lat) / wall, 1),
                              "latency_ms_p50": round(float(np.percentile(ms, 50)), 2),
                              "latency_ms_p99": round(float(np.percentile(ms, 99)), 2),
                              "embed_forwards": fw,
                              "search_launches": (st._batcher.launches - l0) if mode != "fused" else fw,
                              "worker_ms_per_forward": {k: round(1e3 * wt[k] / n, 3) for k in ("launch", "wait", "lists")}
                              if mode == "coalesce" else
                              {k: (round(1e3 * v / max(1, fused.cohorts - c0), 3) if k != "bubbles" else v)
                               for k, v in fused.timing.items()} if mode == "fused" else None,
                              "profiled": bool(a.profile), "untracked_results": bool(a.untracked),
                              "app_gc_freeze": bool(a.gc_freeze),
                              "model": "bge-large shape (random init), bf16", "path": "VectorRetriever.retrieve"}),
                  flush=True)


if __name__ == "__main__":
    main()

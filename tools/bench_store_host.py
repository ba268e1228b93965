#!/usr/bin/env python3
"""Host side of the drop-in store's async search path, without a GPU: HipVectorStore's micro-batcher, native
submit / eventfd completion / collect and _assemble over an index stand-in that answers at once (precomputed rows), so
the figure is the Python work per query -- the part Python's cycle collector competes with.
C client coroutines each issue sequential ``await store.search(query_embedding=q, top_k=k)`` calls and hold the last
answer, as tools/bench_async.py's clients do.  One JSON line per variant.
Usage: python tools/bench_store_host.py [--rows 200000 --clients 256 --seconds 3 --torch 1]"""
from __future__ import annotations

import argparse
import asyncio
import gc
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "youtu-rag_amd"), REPO]

import numpy as np  # noqa: E402


class InstantIndex:
    """search_submit_host answers at once: the completion count goes to the eventfd before the call returns."""

    def __init__(self, n, dim, k):
        self.n, self.dim, self.devices = n, dim, [0]
        rng = np.random.default_rng(0)
        self.rows = rng.integers(0, n, (1024, k)).astype(np.int64)
        self.scores = np.sort(rng.random((1024, k)).astype(np.float32), axis=1)[:, ::-1].copy()
        self.tickets, self.next = {}, 1

    def size(self):
        return self.n, self.n

    def search_submit_host(self, q, k, notify_fd=-1):
        t = self.next
        self.next += 1
        self.tickets[t] = len(q)
        os.eventfd_write(notify_fd, 1)
        return t

    def search_poll(self, ticket):
        return 1

    def search_collect(self, ticket, B, k):
        self.tickets.pop(ticket)
        i = ticket % 512
        return self.scores[i:i + B, :k], self.rows[i:i + B, :k]

    def close(self):
        pass


def build(n, dim, max_batch, k):
    from hiprag.rag import HipVectorStore, VectorStoreConfig

    idx = InstantIndex(n, dim, k)
    cfg = VectorStoreConfig(backend="hip", collection_name="host", persist_directory="/tmp/hiprag_store_host",
                            index_params={"persist": False, "max_batch": max_batch})
    st = HipVectorStore(cfg, index_factory=lambda d: idx)
    st._ensure_index(dim)
    recs = []
    for r in range(n):
        d, i = divmod(r, 1000)
        recs.append({"id": f"doc{d}_chunk_{i}", "document_id": f"doc{d}", "content": "", "chunk_index": i,
                     "metadata": {"document_id": f"doc{d}", "chunk_index": i}})
    st._append_tables(recs, None)
    return st


async def clients(st, qs, C, seconds, k):
    stop = time.perf_counter() + seconds
    done = [0]

    async def client(c):
        j = c
        res = None
        while time.perf_counter() < stop:
            res = await st.search(query_embedding=qs[j % len(qs)], top_k=k)  # (the last answer stays held)
            done[0] += 1
            j += C
        return res

    t0 = time.perf_counter()
    await asyncio.gather(*(client(c) for c in range(C)))
    return done[0] / (time.perf_counter() - t0)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--rows", type=int, default=200_000)
    p.add_argument("--dim", type=int, default=64)
    p.add_argument("--clients", type=int, default=256)
    p.add_argument("--max-batch", type=int, default=64)
    p.add_argument("--seconds", type=float, default=3.0)
    p.add_argument("--k", type=int, default=10)
    p.add_argument("--torch", type=int, default=1, help="import torch first (a serving process's heap)")
    p.add_argument("--freeze", default="0", help="0/1 list: the application calls gc.freeze() after loading")
    p.add_argument("--assemble", default="c", help="c / py: the store's result assembly (_hostfast or the Python loop)")
    a = p.parse_args()
    if a.assemble == "py":
        from hiprag.rag import storage

        storage._hostfast = None
    if a.torch:
        import torch  # noqa: F401
    st = build(a.rows, a.dim, a.max_batch, a.k)
    qs = [list(np.random.default_rng(i).standard_normal(a.dim).astype(np.float32)) for i in range(64)]
    for fz in [int(x) for x in a.freeze.split(",")]:
        gc.collect()
        if fz:
            gc.freeze()
        else:
            gc.unfreeze()
        g0 = [s["collections"] for s in gc.get_stats()]
        qps = asyncio.run(clients(st, qs, a.clients, a.seconds, a.k))
        g1 = [s["collections"] for s in gc.get_stats()]
        print(json.dumps({"freeze": fz, "qps": round(qps, 1), "clients": a.clients, "max_batch": a.max_batch,
                          "tracked_objects": len(gc.get_objects()), "collections_per_gen": [y - x for x, y in zip(g0, g1)],
                          "torch": a.torch, "assemble": a.assemble}), flush=True)


if __name__ == "__main__":
    main()

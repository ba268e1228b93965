"""Filtered search on one GPU: the host entry point (hr_index_search with a row mask, the
HipVectorStore path of a where-clause) at 10M x 1024 bf16, B = 64, top-10, for masks of
different selectivity.  With HIPRAG_TILE_LIST=0 every search scans all tiles (A/B).
Usage: python tools/bench_filter.py [rows]"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "youtu-rag_amd"), REPO]
import numpy as np  # noqa: E402

from hiprag import _native, synth  # noqa: E402


def mask_from_bool(allowed):
    pad = (-len(allowed)) % 64
    return np.packbits(np.concatenate([allowed, np.zeros(pad, bool)]), bitorder="little").view(np.uint64).copy()


def main():
    n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 10_000_000
    D, B, K = 1024, 64, 10
    idx = _native.NativeIndex(D, "bf16", "cosine")
    idx.reserve(n)
    idx.add_synthetic(0, 0, n)
    q, _ = synth.planted_queries(0, n, D, B, qseed=7)
    rng = np.random.default_rng(0)
    cases = {"none": None}
    doc = np.zeros(n, bool)
    doc[n // 3:n // 3 + 10_000] = True  # one document's chunks (contiguous rows)
    cases["1 document (10k rows)"] = doc
    docs = np.zeros(n, bool)
    for lo in rng.choice(n - 2000, 50, replace=False):
        docs[lo:lo + 2000] = True  # 50 documents of 2k chunks
    cases["50 documents (100k rows)"] = docs
    cases["1% random rows"] = rng.random(n) < 0.01
    cases["10% random rows"] = rng.random(n) < 0.10
    cases["30% random rows"] = rng.random(n) < 0.30
    cases["all rows (mask of ones)"] = np.ones(n, bool)
    stats = idx.stats()
    for name, allowed in cases.items():
        m = None if allowed is None else mask_from_bool(allowed)
        for _ in range(2):
            idx.search(q, K, m)
        t0 = time.perf_counter()
        reps = 10
        for _ in range(reps):
            idx.search(q, K, m)
        ms = (time.perf_counter() - t0) / reps * 1e3
        frac = 1.0 if allowed is None else float(np.mean(allowed))
        tot, mx = idx.last_candidates()
        st0 = stats
        stats = idx.stats()
        fails = stats["guard_failures"] - st0["guard_failures"]
        print(f"{name:28s} allowed {frac:7.4f}  {ms:8.3f} ms/batch  {B / ms * 1e3:10.0f} QPS  "
              f"candidates/query {tot / B:8.0f} (max {mx})  guard failures {fails} / {12 * B}", flush=True)


def pipelined(n=10_000_000):
    """The same masks through the pipelined device path (ShardedSearch, device mask: the tile list
    is built on the GPU), 20 batches in flight two deep."""
    import torch

    from hiprag.dist import ShardedSearch

    D, B, K, nb = 1024, 64, 10, 20
    idx = _native.NativeIndex(D, "bf16", "cosine")
    idx.reserve(n)
    idx.add_synthetic(0, 0, n)
    qs = torch.from_numpy(np.stack([synth.planted_queries(0, n, D, B, qseed=100 + i)[0] for i in range(nb)])).cuda()
    ready = torch.cuda.Event()
    ready.record()
    ss = ShardedSearch(idx, 0, max_batch=B)
    rng = np.random.default_rng(1)
    doc = np.zeros(n, bool)
    doc[n // 3:n // 3 + 10_000] = True
    for name, allowed in (("none", None), ("1 document (10k rows)", doc), ("1% random rows", rng.random(n) < 0.01)):
        mp = 0
        if allowed is not None:
            md = torch.from_numpy(mask_from_bool(allowed).view(np.int64)).cuda()
            mp = md.data_ptr()
        for i in range(3):
            ss.submit(qs[i], K, mask_ptr=mp, q_ready=ready)
        ss.finalize_all()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(nb):
            ss.submit(qs[i], K, mask_ptr=mp, q_ready=ready)
        ss.finalize_all()
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / nb * 1e3
        print(f"pipelined {name:28s} {ms:8.3f} ms/batch  {B / ms * 1e3:10.0f} QPS", flush=True)


def store(n=10_000_000):
    """Where-clauses through the drop-in store: HipVectorStore.search_batch(filters=...) at n rows of
    1000-chunk documents (+ one summary row each), the filters kb_file_search / kb_embedding_search
    build.  Reports the where -> bitmap compile time (first call, then cached) and the end-to-end
    search time per 64-query batch."""
    from hiprag.rag import HipVectorStore, VectorStoreConfig
    from hiprag.rag import filters as F

    D, B, K = 1024, 64, 10
    idx = _native.NativeIndex(D, "bf16", "cosine")
    idx.reserve(n)
    idx.add_synthetic(0, 0, n)
    cfg = VectorStoreConfig(backend="hip", collection_name="bench", persist_directory="/tmp/hiprag_bench",
                            index_params={"dtype": "bf16", "persist": False})
    st = HipVectorStore(cfg, index_factory=lambda d: idx)
    st._ensure_index(D)
    t0 = time.perf_counter()
    recs = []
    for r in range(n):
        d, i = divmod(r, 1000)
        recs.append({"id": f"doc{d}_chunk_{i}", "document_id": f"doc{d}", "content": "", "chunk_index": i,
                     "metadata": {"document_id": f"doc{d}", "chunk_index": i, "source": f"file_{d % 5000}.pdf",
                                  "index_type": "index_summary" if i == 999 else "index_content"}})
        if len(recs) == 1_000_000:
            st._append_tables(recs, None)
            recs = []
    if recs:
        st._append_tables(recs, None)
    print(f"host tables for {n} rows in {time.perf_counter() - t0:.1f}s", flush=True)
    q, _ = synth.planted_queries(0, n, D, B, qseed=7)
    cases = [("none", None), ("index_type == index_summary (kb_file_search)", {"index_type": {"$eq": "index_summary"}}),
             ("source $in 2 files", {"source": {"$in": ["file_17.pdf", "file_4000.pdf"]}}),
             ("document_id == doc777", {"document_id": "doc777"}),
             ("summary AND source $in", {"$and": [{"source": {"$in": ["file_1.pdf", "file_2.pdf"]}},
                                                  {"index_type": {"$eq": "index_summary"}}]}),
             ("chunk_index < 500 (dense)", {"chunk_index": {"$lt": 500}})]
    for name, f in cases:
        t0 = time.perf_counter()
        if f:
            F.evaluate_words(f, st._cols)
        first = (time.perf_counter() - t0) * 1e3
        t0 = time.perf_counter()
        if f:
            for _ in range(10):
                F.evaluate_words(f, st._cols)
        cached = (time.perf_counter() - t0) * 1e3 / 10
        st.search_batch(q, K, f)
        t0 = time.perf_counter()
        for _ in range(10):
            res = st.search_batch(q, K, f)
        ms = (time.perf_counter() - t0) * 1e3 / 10
        print(f"store {name:46s} compile first {first:7.2f} ms, cached {cached:6.3f} ms; search_batch {ms:8.3f} "
              f"ms/batch ({sum(len(r) for r in res) / B:.1f} hits/query)", flush=True)


if __name__ == "__main__":
    if os.environ.get("STORE") == "1":
        store(int(float(sys.argv[1])) if len(sys.argv) > 1 else 10_000_000)
        sys.exit(0)
    if os.environ.get("PIPELINED") == "1":
        pipelined(int(float(sys.argv[1])) if len(sys.argv) > 1 else 10_000_000)
        sys.exit(0)
    main()

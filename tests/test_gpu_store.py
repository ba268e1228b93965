"""GPU: the full drop-in stack -- HipVectorStore on libhiprag.so behind the reference's
VectorRetriever semantics -- reproduces the golden retriever outputs; persistence round-trips."""
import asyncio
import json
import os

import numpy as np
import pytest

from hiprag.rag import (BatchedVectorRetriever, Chunk, HipVectorStore, RetrieverConfig, VectorRetriever,
                        VectorStoreConfig, VectorStoreFactory)

pytestmark = pytest.mark.gpu


class TableEmbedder:
    def __init__(self, table):
        self.table = table

    async def embed_query(self, q):
        return self.table[q].tolist()

    async def embed_texts(self, texts):
        return [self.table[t].tolist() for t in texts]


def _chunks(d, meta):
    return [Chunk(id=f"chunk_{r}", document_id=m["document_id"], content=f"text {r}", chunk_index=m["chunk_index"],
                  metadata={"group": m["group"]}, embedding=d["corpus"][r].tolist()) for r, m in enumerate(meta["metas"])]


@pytest.mark.parametrize("dtype", [None, "f32", "bf16"])
def test_store_retriever_golden(tmp_path, golden_dir, dtype):
    """dtype None: no index_params dtype -- the store's default must be fp32, what the reference stores
    (faiss_store.py:98; Chroma float32), so the golden ranks and scores are reproduced exactly."""
    d = dict(np.load(os.path.join(golden_dir, "c1_retrieval.npz")))
    meta = json.load(open(os.path.join(golden_dir, "c1_retrieval.json")))
    cfg = VectorStoreConfig(backend="hip", collection_name="c1", persist_directory=str(tmp_path),
                            index_params={} if dtype is None else {"dtype": dtype})
    store = VectorStoreFactory.create(cfg)
    assert isinstance(store, HipVectorStore)
    if dtype is None:
        assert store.dtype == "f32"
        dtype = "f32"
    asyncio.run(store.add_chunks(_chunks(d, meta)))
    emb = TableEmbedder(dict(zip(meta["query_names"], d["queries"])))
    for tag, rc, kw in [("thr0", RetrieverConfig(top_k=5, similarity_threshold=0.0), {}),
                        ("thr_default", RetrieverConfig(top_k=5), {}),
                        ("filtered_g1", RetrieverConfig(top_k=5, similarity_threshold=0.0), {"filters": {"group": "g1"}})]:
        for cls in (VectorRetriever, BatchedVectorRetriever):
            got = asyncio.run(cls(store, emb, rc).batch_retrieve(meta["query_names"], top_k=5, **kw))
            exp = meta["results"][tag]
            if dtype == "f32":  # the golden store is fp32; bf16 storage may legitimately reorder near-ties
                assert [[(r.chunk.id, r.rank) for r in res] for res in got] == \
                    [[(e["chunk_id"], e["rank"]) for e in res] for res in exp]
                for res, ex in zip(got, exp):
                    np.testing.assert_allclose([r.score for r in res], [e["score"] for e in ex], atol=1e-5, rtol=0)
            else:
                assert [res[0].chunk.id for res in got if res] == [res[0]["chunk_id"] for res in exp if res]
    # persistence: a new store object on the same directory serves the same answers
    before = store.search_batch(d["queries"], 5)
    store2 = HipVectorStore(cfg)
    assert asyncio.run(store2.count()) == 1000
    after = store2.search_batch(d["queries"], 5)
    assert [[c.id for c, _ in res] for res in before] == [[c.id for c, _ in res] for res in after]
    asyncio.run(store2.delete_by_document_id("doc_0"))
    assert asyncio.run(HipVectorStore(cfg).count()) == 990


def test_euclidean_store_vs_oracle(tmp_path, golden_dir):
    """distance_metric="euclidean" through the whole store: Chroma's l2 similarity 1 - |q - x|^2
    (chroma_store.py:48-53, :135), exact ids and bits of the oracle."""
    import oracle
    from oracle import ref_numpy as R

    d = dict(np.load(os.path.join(golden_dir, "c1_retrieval.npz")))
    meta = json.load(open(os.path.join(golden_dir, "c1_retrieval.json")))
    cfg = VectorStoreConfig(backend="hip", collection_name="c1l2", persist_directory=str(tmp_path),
                            distance_metric="euclidean", index_params={"dtype": "f32"})
    store = VectorStoreFactory.create(cfg)
    asyncio.run(store.add_chunks(_chunks(d, meta)))
    s_ref, r_ref = oracle.c_search(R.process_rows(d["corpus"], "l2", "f32"), "f32", d["queries"], 5, metric="l2")
    for b, q in enumerate(d["queries"]):
        res = asyncio.run(store.search(query_embedding=q.tolist(), top_k=5))
        assert [c.id for c, _ in res] == [f"chunk_{x}" for x in r_ref[b]]
        np.testing.assert_array_equal(np.array([s for _, s in res], np.float32), s_ref[b].astype(np.float32))


def test_store_native_async_concurrent_vs_oracle(tmp_path):
    """The reference's call pattern on the device: many concurrent single-query store.search calls
    (VectorRetriever.retrieve, base_retriever.py:58-63).  Unfiltered batches are launched from the event
    loop through hr_index_search_submit_host (completion by eventfd, no worker thread); every answer is
    the oracle's, filtered ones (worker path) too, and a clear with batches in flight resolves them empty."""
    import oracle
    from oracle import ref_numpy as R

    rng = np.random.default_rng(21)
    n, dim = 20_000, 256
    raw = R.gen_rows(5, 0, n, dim)
    cfg = VectorStoreConfig(backend="hip", collection_name="asy", persist_directory=str(tmp_path),
                            index_params={"dtype": "bf16", "persist": False, "max_batch": 32})
    store = HipVectorStore(cfg)
    store.add_chunks_sync([Chunk(id=f"c{i}", document_id=f"d{i // 100}", content=str(i), chunk_index=i % 100,
                                 metadata={"grp": f"g{i % 3}"}, embedding=raw[i].tolist()) for i in range(n)])
    q = (raw[rng.choice(n, 200, replace=False)] + 300.0 * rng.standard_normal((200, dim))).astype(np.float32)
    stored = R.process_rows(raw, "cosine", "bf16")
    s_ref, r_ref = oracle.c_search(stored, "bf16", R.process_queries(q, "cosine"), 10)
    allowed = np.arange(n) % 3 == 1
    sf_ref, rf_ref = oracle.c_search(stored, "bf16", R.process_queries(q[:40], "cosine"), 5,
                                     oracle.mask_from_bool(allowed))

    async def main():
        un = [store.search(query_embedding=x.tolist(), top_k=10) for x in q]
        fi = [store.search(query_embedding=x.tolist(), top_k=5, filters={"grp": "g1"}) for x in q[:40]]
        return await asyncio.gather(*un, *fi)

    out = asyncio.run(main())
    assert store._batcher.native_launches >= 200 // 32
    for b in range(200):
        assert [c.id for c, _ in out[b]] == [f"c{r}" for r in r_ref[b]]
        np.testing.assert_array_equal(np.array([s for _, s in out[b]], np.float32), s_ref[b].astype(np.float32))
    for b in range(40):
        assert [c.id for c, _ in out[200 + b]] == [f"c{r}" for r in rf_ref[b]]

    async def clear_mid_flight():
        tasks = [asyncio.ensure_future(store.search(query_embedding=x.tolist(), top_k=3)) for x in q[:64]]
        await asyncio.sleep(0)
        await asyncio.sleep(0)
        await store.clear()
        return await asyncio.gather(*tasks)

    res = asyncio.run(clear_mid_flight())
    assert all(r == [] or len(r) == 3 for r in res)  # finished before the clear, or emptied by it
    store.close()

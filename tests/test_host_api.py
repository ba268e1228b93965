"""CPU: the host mirror of the reference plugin API (hiprag.rag) reproduces the
reference's retriever/store/chunker/embedder behaviour.  The device index is replaced
by the oracle-backed tests/fake_index.OracleIndex (host-logic tests only; the HIP path
is covered by the -m gpu suite)."""
import asyncio
import base64
import json
import os

import numpy as np
import pytest

from fake_index import OracleIndex
from hiprag.rag import (BatchedVectorRetriever, Chunk, ChunkingConfig, HipVectorStore, RecursiveTextSplitter,
                        RetrieverConfig, ServiceEmbedder, VectorRetriever, VectorStoreConfig, VectorStoreFactory)
from hiprag.rag import embeddings as E
from hiprag.rag import filters as F


def run(coro):
    return asyncio.run(coro)


class TableEmbedder:
    def __init__(self, table):
        self.table = table
        self.calls = 0

    async def embed_query(self, q):
        self.calls += 1
        return self.table[q].tolist()

    async def embed_texts(self, texts):
        return [self.table[t].tolist() for t in texts]


def make_store(tmp_path, dtype="f32", persist=False, metric="cosine"):
    cfg = VectorStoreConfig(backend="hip", collection_name="kb", persist_directory=str(tmp_path),
                            distance_metric=metric, index_params={"dtype": dtype, "persist": persist})
    return HipVectorStore(cfg, index_factory=lambda dim: OracleIndex(dim, dtype, "ip" if metric == "dot" else metric))


@pytest.fixture(scope="module")
def c1(golden_dir):
    d = dict(np.load(os.path.join(golden_dir, "c1_retrieval.npz")))
    meta = json.load(open(os.path.join(golden_dir, "c1_retrieval.json")))
    return d, meta


def _c1_store(tmp_path, c1, dtype="f32"):
    d, meta = c1
    store = make_store(tmp_path, dtype)
    chunks = [Chunk(id=f"chunk_{r}", document_id=m["document_id"], content=f"text {r}", chunk_index=m["chunk_index"],
                    metadata={"group": m["group"], "empty": None}, embedding=d["corpus"][r].tolist())
              for r, m in enumerate(meta["metas"])]
    run(store.add_chunks(chunks[:600]))
    run(store.add_chunks(chunks[600:]))
    return store


@pytest.mark.parametrize("retriever_cls", [VectorRetriever, BatchedVectorRetriever])
def test_retriever_matches_reference_golden(tmp_path, c1, retriever_cls):
    d, meta = c1
    store = _c1_store(tmp_path, c1)
    emb = TableEmbedder(dict(zip(meta["query_names"], d["queries"])))
    for tag, cfg, kw in [("thr0", RetrieverConfig(top_k=5, similarity_threshold=0.0), {}),
                         ("thr_default", RetrieverConfig(top_k=5), {}),
                         ("filtered_g1", RetrieverConfig(top_k=5, similarity_threshold=0.0), {"filters": {"group": "g1"}})]:
        ret = retriever_cls(vector_store=store, embedder=emb, config=cfg)
        got = run(ret.batch_retrieve(meta["query_names"], top_k=5, **kw))
        exp = meta["results"][tag]
        assert [[(r.chunk.id, r.rank) for r in res] for res in got] == [[(e["chunk_id"], e["rank"]) for e in res]
                                                                         for res in exp]
        for res, ex in zip(got, exp):
            np.testing.assert_allclose([r.score for r in res], [e["score"] for e in ex], atol=1e-5, rtol=0)


def test_batched_retriever_uses_one_search(tmp_path, c1):
    d, meta = c1
    store = _c1_store(tmp_path, c1)
    emb = TableEmbedder(dict(zip(meta["query_names"], d["queries"])))
    before = store._index.searches
    run(BatchedVectorRetriever(store, emb, RetrieverConfig(top_k=3)).batch_retrieve(meta["query_names"]))
    assert store._index.searches - before == 1


def test_store_semantics(tmp_path, c1):
    store = _c1_store(tmp_path, c1)
    assert run(store.count()) == 1000
    # chroma metadata convention: document_id/chunk_index merged in, None values dropped
    ch = run(store.get_by_id("chunk_7"))
    assert ch.metadata == {"document_id": "doc_0", "chunk_index": 7, "group": "g3"}
    assert ch.embedding is not None and len(ch.embedding) == 128
    assert run(store.get_by_id("nope")) is None
    # existing ids are skipped, duplicates inside one call rejected
    run(store.add_chunks([Chunk(id="chunk_7", document_id="x", content="y", chunk_index=0, embedding=[1.0] * 128)]))
    assert run(store.count()) == 1000
    with pytest.raises(ValueError):
        run(store.add_chunks([Chunk(id="a", document_id="x", content="", chunk_index=0, embedding=[1.0] * 128)] * 2))
    with pytest.raises(ValueError):
        run(store.add_chunks([Chunk(id="b", document_id="x", content="", chunk_index=0, embedding=[1.0] * 7)]))
    # deletes
    assert run(store.delete_by_document_id("doc_3")) == 10
    assert run(store.delete_by_document_id("doc_3")) == 0
    run(store.delete(["chunk_0", "chunk_1", "missing"]))
    assert run(store.count()) == 988
    assert run(store.delete_by_metadata({"group": "g2", "document_id": "doc_5"})) == 3  # rows 50, 54, 58
    q = np.asarray(run(store.get_by_id("chunk_45")).embedding)
    hits = run(store.search(query_embedding=q.tolist(), top_k=5))
    assert all(c.document_id != "doc_3" for c, _ in hits)
    assert hits[0][0].id == "chunk_45" and abs(hits[0][1] - 1.0) < 1e-5
    # top_k has no cap (Chroma n_results): beyond HR_MAX_K and beyond the live count
    many = run(store.search(query_embedding=q.tolist(), top_k=300))
    assert len(many) == 300 and [c.id for c, _ in many[:5]] == [c.id for c, _ in hits]
    assert len(run(store.search(query_embedding=q.tolist(), top_k=5000))) == run(store.count())
    assert run(store.search(query_embedding=q.tolist(), top_k=0)) == []
    run(store.clear())
    assert run(store.count()) == 0 and run(store.search([0.0] * 128)) == []


def test_store_persistence_roundtrip(tmp_path, monkeypatch):
    # the HIP index files are exercised on the GPU (test_gpu_store.py); here the row tables
    store = make_store(tmp_path, persist=False)
    run(store.add_chunks([Chunk(id=f"c{i}", document_id="d", content=str(i), chunk_index=i, embedding=[float(i), 1.0])
                          for i in range(5)]))
    assert store.search_batch([[1.0, 0.0], [0.0, 1.0]], top_k=2)[0][0][0].id == "c4"


def test_factory_and_config():
    cfg = VectorStoreConfig()
    assert cfg.backend == "chroma" and cfg.distance_metric == "cosine"
    with pytest.raises(ValueError):
        VectorStoreFactory.create(cfg.model_copy(update={"backend": "milvus"}))
    assert "***" in repr(VectorStoreConfig(api_key="secret")) and "secret" not in repr(VectorStoreConfig(api_key="secret"))
    # distance_metric -> index metric (chroma_store.py:48-53: euclidean = hnsw "l2", dot = "ip")
    assert HipVectorStore(VectorStoreConfig(distance_metric="euclidean", index_params={"persist": False}),
                          index_factory=lambda d: None).metric == "l2"
    assert HipVectorStore(VectorStoreConfig(distance_metric="dot", index_params={"persist": False}),
                          index_factory=lambda d: None).metric == "ip"


def test_euclidean_store_semantics():
    """euclidean: similarity = 1 - squared L2 distance (Chroma l2 space, chroma_store.py:48-53, :135),
    nearest rows first, raw (unnormalised) vectors."""
    store = HipVectorStore(VectorStoreConfig(distance_metric="euclidean", index_params={"persist": False,
                                                                                            "dtype": "f32"}),
                           index_factory=lambda d: OracleIndex(d, "f32", "l2"))
    vecs = [[0.0, 0.0], [1.0, 0.0], [3.0, 4.0], [0.5, 0.5]]
    asyncio.run(store.add_chunks([Chunk(id=f"e{i}", content=str(i), document_id="d", chunk_index=i, embedding=v)
                                  for i, v in enumerate(vecs)]))
    res = asyncio.run(store.search(query_embedding=[1.0, 0.0], top_k=3))
    assert [c.id for c, _ in res] == ["e1", "e3", "e0"]
    np.testing.assert_allclose([s for _, s in res], [1.0, 0.5, 0.0])


def test_chunker_golden(golden_dir):
    g = json.load(open(os.path.join(golden_dir, "chunker.json")))
    for case in g["cases"]:
        sp = RecursiveTextSplitter(ChunkingConfig(chunk_size=case["chunk_size"], chunk_overlap=case["chunk_overlap"]))
        for text, expected in zip(g["texts"], case["chunks"]):
            assert sp.split_text(text) == expected


def test_service_embedder_wire_golden(golden_dir, monkeypatch):
    g = json.load(open(os.path.join(golden_dir, "service_embedder.json")))
    table = {t: np.asarray(v, np.float32) for t, v in zip(g["texts"], g["embeddings"])}
    calls = []

    def fake_post(url, body, timeout=60, max_retries=3, retry_delay=2.0):
        route = url.rsplit("/", 1)[-1]
        calls.append({"url": route, "n": len(body.get("docs", [body.get("query")]))})
        arr = (np.stack([table[t] for t in body["docs"]]) if "docs" in body
               else np.asarray(g["query_embedding"], np.float32))
        return {"embedding": base64.b64encode(arr.tobytes()).decode("ascii"), "shape": list(arr.shape)}

    monkeypatch.setattr(E, "post_with_retry", fake_post)
    emb = ServiceEmbedder("http://embed.invalid:8081/", batch_size=g["batch_size"], check_health=False)
    assert emb.service_url == "http://embed.invalid:8081"
    vecs = run(emb.embed_texts(g["texts"]))
    qv = run(emb.embed_query(g["query"]))
    assert calls == g["calls"]
    assert vecs == g["embeddings"] and qv == g["query_embedding"]


def test_filters_chroma_semantics():
    cols = F.MetadataColumns()
    cols.append([{"a": 1, "s": "x", "b": True}, {"a": 5, "s": "y"}, {"s": "x", "b": 1}, {"a": 3.5, "s": "z"}])
    ev = lambda w: F.evaluate(w, cols).tolist()  # noqa: E731
    assert ev({"s": "x"}) == [True, False, True, False]
    assert ev({"s": {"$ne": "x"}}) == [False, True, False, True]
    assert ev({"a": {"$gte": 3.5}}) == [False, True, False, True]
    assert ev({"a": {"$lt": 5, "$gt": 1}}) == [False, False, False, True]
    assert ev({"s": {"$in": ["y", "z"]}}) == [False, True, False, True]
    assert ev({"s": {"$nin": ["y", "z"]}}) == [True, False, True, False]
    assert ev({"$and": [{"s": "x"}, {"a": 1}]}) == [True, False, False, False]
    assert ev({"$or": [{"s": "y"}, {"a": {"$lte": 1}}]}) == [True, True, False, False]
    assert ev({"b": True}) == [True, False, False, False]  # True does not match 1
    assert ev({"missing": {"$ne": 3}}) == [False] * 4
    with pytest.raises(ValueError):
        ev({"a": {"$regex": "x"}})
    bm = F.to_bitmap(np.array([True, False] * 40))
    assert bm.dtype == np.uint64 and len(bm) == 2 and int(bm[0]) == int("01" * 32, 2)

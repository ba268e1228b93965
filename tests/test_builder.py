"""KnowledgeBuilder and CourseSearcher (hiprag.rag.builder, SURVEY §8(b) callers) against
tests/golden/builder.json, which the REFERENCE's own base_builder.py / chroma_retrical_text2sql.py produced
(tests/golden/gen_builder.py): build statuses (incl. the per-document error of a poisoned text), the
md5 chunk ids and metadata the store received in order, rebuild clearing, the embedder / store factory
calls, and every CourseSearcher result list (ids, metadata, scores) equal.  CPU: oracle-backed fake
index; GPU: libhiprag.so."""
import asyncio
import json
import os

import pytest

from fake_index import OracleIndex
from hash_embed import HashEmbedder
from hiprag.rag import Document, HipVectorStore, VectorStoreConfig
from hiprag.rag import builder as B
from hiprag.rag import storage as S
from hiprag.rag.config import KnowledgeBuilderConfig


@pytest.fixture(scope="module")
def golden(golden_dir):
    return json.load(open(os.path.join(golden_dir, "builder.json")))


def _docs(ds):
    return [Document(id=d["id"], content=d["content"], metadata=dict(d["metadata"])) for d in ds]


def _ids(store):
    return [r[0] for r in store._records if r is not None]


def _run(golden, tmp_path, monkeypatch, device: bool):
    emb_calls, store_calls = [], []

    def embedder_create(backend="auto", **kw):
        emb_calls.append({"backend": backend, **kw})
        return HashEmbedder(batch_size=kw.get("batch_size") or 16)

    monkeypatch.setattr(B.EmbedderFactory, "create", staticmethod(embedder_create))
    cfg = VectorStoreConfig(collection_name="t2s_collection", persist_directory=str(tmp_path / "s"),
                            index_params={"dtype": "f32", "persist": False})
    store = HipVectorStore(cfg) if device else HipVectorStore(cfg, index_factory=lambda d: OracleIndex(d, "f32"))

    kb = B.KnowledgeBuilder(store, KnowledgeBuilderConfig(**golden["kb_config"]))
    calls = {"build_a": lambda: kb.build_from_documents(_docs(golden["docs"]["a"])),
             "add_b": lambda: kb.add_documents(_docs(golden["docs"]["b"])),
             "rebuild_c": lambda: kb.build_from_documents(_docs(golden["docs"]["c"]), rebuild=True)}
    steps = {s["step"]: s for s in golden["steps"]}
    for name in ("build_a", "add_b"):
        st = asyncio.run(calls[name]())
        assert {k: getattr(st, k) for k in steps[name]["status"]} == steps[name]["status"], name
        assert _ids(store) == steps[name]["store_ids"], name
        assert asyncio.run(kb.get_build_status()) is st
    snap = [{"id": r["id"], "content": r["content"], "metadata": r["metadata"]}
            for r in map(store.record, range(len(store._records))) if r is not None]
    assert snap == golden["store_after_add_b"]

    for k, v in golden["env"].items():
        monkeypatch.setenv(k, v)
    monkeypatch.chdir(tmp_path)  # no configs/ here: the env-default path, as in the fixture

    def store_create(c, **kw):
        store_calls.append({"backend": c.backend, "collection_name": c.collection_name,
                            "persist_directory": c.persist_directory, "distance_metric": c.distance_metric})
        return store

    monkeypatch.setattr(S.VectorStoreFactory, "create", staticmethod(store_create))
    cs = B.CourseSearcher(collection_name="t2s_collection")
    for case in golden["course_searches"]:
        got = asyncio.run(cs.search(case["query"], top_k=case["top_k"], filter_conditions=case["filter_conditions"]))
        assert json.loads(json.dumps(got)) == case["results"], case["query"]
    assert len(cs._embedding_cache) == golden["embedding_cache_size"]
    # the batched form gives the same lists (one embedder batch, one index launch per filter)
    cs.clear_embedding_cache()
    for case in golden["course_searches"]:
        got = asyncio.run(cs.search_batch([case["query"], case["query"]], top_k=case["top_k"],
                                          filter_conditions=case["filter_conditions"]))
        assert json.loads(json.dumps(got)) == [case["results"]] * 2
    assert emb_calls == golden["embedder_factory_calls"]
    assert store_calls == golden["store_factory_calls"]

    st = asyncio.run(calls["rebuild_c"]())
    assert {k: getattr(st, k) for k in steps["rebuild_c"]["status"]} == steps["rebuild_c"]["status"]
    assert _ids(store) == steps["rebuild_c"]["store_ids"]
    return store


def test_builder_and_course_searcher_match_reference_host(golden, tmp_path, monkeypatch):
    _run(golden, tmp_path, monkeypatch, device=False)


def test_builder_batches_across_documents_and_attributes_failures(golden, tmp_path):
    """Embedder batches span documents; a batch holding the poisoned document is retried per document."""
    cfg = VectorStoreConfig(collection_name="x", persist_directory=str(tmp_path / "x"),
                            index_params={"dtype": "f32", "persist": False})
    store = HipVectorStore(cfg, index_factory=lambda d: OracleIndex(d, "f32"))
    emb = HashEmbedder(batch_size=64)
    kb = B.KnowledgeBuilder(store, KnowledgeBuilderConfig(**golden["kb_config"]), embedder=emb)
    st = asyncio.run(kb.build_from_documents(_docs(golden["docs"]["a"])))
    assert st.status == "completed" and len(st.errors) == 1 and "adoc3" in st.errors[0]
    assert _ids(store) == golden["steps"][0]["store_ids"]
    assert len(emb.calls) < len(golden["docs"]["a"]) + 2  # packed batches + the per-document retry


def test_builder_failure_status(tmp_path):
    class Broken:
        async def clear(self):
            raise RuntimeError("store offline")

    kb = B.KnowledgeBuilder(Broken(), KnowledgeBuilderConfig(), embedder=HashEmbedder())
    with pytest.raises(RuntimeError):
        asyncio.run(kb.build_from_documents([], rebuild=True))
    st = asyncio.run(kb.get_build_status())
    assert st.status == "failed" and st.errors == ["store offline"] and st.end_time


@pytest.mark.gpu
def test_builder_and_course_searcher_match_reference_device(golden, tmp_path, monkeypatch):
    _run(golden, tmp_path, monkeypatch, device=True)

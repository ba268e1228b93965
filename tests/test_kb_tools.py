"""The KB-search tools (hiprag.rag.kb_tools) against tests/golden/kb_tools.json,
which the REFERENCE's own KBSearchToolkit produced (tests/golden/gen_kb_tools.py): every tool call's
JSON string byte-identical, the RetrieverConfig that _create_retriever builds, the per-collection
store cache.  CPU: the device index is the oracle-backed fake (host logic); GPU: the real
HipVectorStore through libhiprag.so."""
import asyncio
import json
import os

import numpy as np
import pytest

from fake_index import OracleIndex
from hiprag.rag import Chunk, HipVectorStore
from hiprag.rag import kb_tools as K
from oracle import ref_numpy as R


class TableEmbedder:
    def __init__(self, table):
        self.table = table

    async def embed_query(self, q):
        return self.table[q]


@pytest.fixture(scope="module")
def golden(golden_dir):
    return json.load(open(os.path.join(golden_dir, "kb_tools.json")))


def _failing_reranker(backend):
    raise RuntimeError(f"reranker backend {backend!r} unreachable offline")


def _run(golden, tmp_path, monkeypatch, device: bool):
    monkeypatch.setattr(K, "_reranker_from", _failing_reranker)
    rows = golden["rows"]
    vecs = R.gen_rows(golden["vectors_seed"], 0, len(rows), golden["dim"])
    kb_table = {int(k): tuple(v) for k, v in golden["kb_table"].items()}
    for run in golden["runs"]:
        calls = []

        def factory(cfg):
            calls.append({"backend": cfg.backend, "persist_directory": cfg.persist_directory,
                          "collection_name": cfg.collection_name, "distance_metric": cfg.distance_metric})
            cfg = cfg.model_copy(update={"persist_directory": str(tmp_path / cfg.collection_name),
                                         "index_params": {"dtype": "f32", "persist": False}})
            if device:
                return HipVectorStore(cfg)
            return HipVectorStore(cfg, index_factory=lambda d: OracleIndex(d, "f32"))

        tk = K.KBSearchToolkit(config=run["toolkit_config"], kb_resolver=kb_table.get, store_factory=factory)
        tk._embedder_cache = TableEmbedder(golden["queries"])
        # the KB contents: each collection filled through add_chunks (chunks + summary vectors)
        for kb, (coll, _) in kb_table.items():
            store = tk._get_or_create_vector_store(coll, run["toolkit_config"].get("vector_store", {}).get(
                "persist_directory", "./rag_data/vector_store"))
            sel = [(r, vecs[r["vec"]]) for r in rows if r["kb"] == kb]
            asyncio.run(store.add_chunks([Chunk(id=r["id"], document_id=r["document_id"], content=r["content"],
                                                chunk_index=r["chunk_index"], metadata=dict(r["metadata"]),
                                                embedding=v.tolist()) for r, v in sel]))
        for o in run["outputs"]:
            got = asyncio.run(getattr(tk, o["tool"])(**o["kwargs"]))
            if "error" in json.loads(o["json"]):  # error path: same shape (the message is Python's)
                assert json.loads(got).keys() == json.loads(o["json"]).keys(), (o["kwargs"], got)
                continue
            assert got == o["json"], (o["tool"], o["kwargs"])
        ret = asyncio.run(tk._create_retriever(1, 7))
        assert {"top_k": ret.config.top_k, "similarity_threshold": ret.config.similarity_threshold,
                "enable_reranking": ret.config.enable_reranking,
                "reranker": ret.reranker is not None} == run["create_retriever"]
        assert calls == run["store_factory_calls"]  # one store per collection, cached
        for case in run["metadata_filters"]:
            assert tk._build_metadata_filters(case["in"]) == case["out"]


def test_kb_tools_match_reference_host(golden, tmp_path, monkeypatch):
    _run(golden, tmp_path, monkeypatch, device=False)


@pytest.mark.gpu
def test_kb_tools_match_reference_gpu(golden, tmp_path, monkeypatch):
    _run(golden, tmp_path, monkeypatch, device=True)


def test_kb_rerank_keeps_the_reference_quirk(golden):
    """kb_rerank passes top_n= to rerank() (kb_search_toolkit.py:391-393): the error JSON."""
    class Rr:
        async def rerank(self, query, results, top_k=None):
            return results

    tk = K.KBSearchToolkit(config={})
    tk.reranker = Rr()
    cands = golden["runs"][0]["outputs"][0]["json"]
    out = json.loads(asyncio.run(tk.kb_rerank("q0", cands)))
    assert "error" in out and "top_n" in out["error"]
    assert asyncio.run(tk.kb_rerank("q", json.dumps({"results": []}))) == json.dumps({"results": []})
    assert "error" in json.loads(asyncio.run(tk.kb_rerank("q", "{not json")))

"""Golden fixtures for the two remaining callers of the search path (SURVEY §8(b) "Callers"), from the
REFERENCE's own code:
  KnowledgeBuilder  utu/rag/knowledge_builder/base_builder.py:17-182 (build_from_documents, add_documents,
                    md5 chunk ids, chunk metadata, per-document error accounting, one add_chunks call)
  CourseSearcher    utu/rag/knowledge_retrieval/chroma_retrical_text2sql.py:45-196 (config fallback,
                    store / embedder construction, embedding cache, filter_conditions -> where, result dicts)

Runs only in the build container (reference tree read-only, no bytecode written).  Both modules are
loaded from their source files and run as written.  Imports that need packages absent here are
registered as small modules first, each standing in for a plug-in point, never for code under test:
  utu.rag.embeddings.factory  EmbedderFactory -> tests/hash_embed.HashEmbedder (records the call)
  utu.rag.storage             VectorStoreFactory -> the FAISS-semantics oracle store with Chroma's
                              conventions (gen_kb_tools.ChromaLikeOracleStore, + clear()) (records the call)
  utu.config.ConfigLoader     load_toolkit_config raises (no configs/ dir offline -> env defaults path)
  utu.utils.log               get_logger = logging.getLogger
Output: builder.json (inputs: documents; expected: build statuses, the chunks the store received, the
factory calls, CourseSearcher results).
"""
from __future__ import annotations

import asyncio
import importlib.util
import json
import logging
import os
import sys
import types

sys.dont_write_bytecode = True
REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(HERE))  # tests/ (hash_embed)

import numpy as np  # noqa: E402

from gen_golden import load_reference  # noqa: E402
from gen_kb_tools import ChromaLikeOracleStore  # noqa: E402
from hash_embed import HashEmbedder  # noqa: E402

WORDS = ("schema table column revenue region quarter student course grade teacher campus enrolment "
         "credit semester faculty budget invoice order customer product warehouse shipment").split()


def documents(seed: int, n: int, tag: str):
    rng = np.random.default_rng(seed)
    docs = []
    for i in range(n):
        n_par = int(rng.integers(0, 6))
        pars = []
        for _ in range(n_par):
            sents = [" ".join(rng.choice(WORDS, int(rng.integers(4, 18)))).capitalize() + "."
                     for _ in range(int(rng.integers(1, 7)))]
            pars.append(" ".join(sents))
        content = "\n\n".join(pars)
        if i == 3:
            content += "\n\nPOISON paragraph the embedding service rejects."
        meta = {"source": f"{tag}_{i}.md", "title": f"t{i % 3}", "page": int(i), "year": 2020 + i % 4,
                "note": None if i % 2 else "n"}
        docs.append({"id": f"{tag}doc{i}", "content": content, "metadata": meta})
    return docs


class Store(ChromaLikeOracleStore):
    async def clear(self):
        self.ids, self.docs, self.metas, self.vecs = [], [], [], []


def status(s):
    return {"status": s.status, "total_documents": s.total_documents, "processed_documents": s.processed_documents,
            "total_chunks": s.total_chunks, "errors": list(s.errors)}


def main():
    mods = load_reference()
    base, config = mods["base"], mods["config"]
    emb_calls, store_calls = [], []
    stores = {}

    class EmbedderFactory:
        @staticmethod
        def create(backend="auto", **kw):
            emb_calls.append({"backend": backend, **kw})
            return HashEmbedder(batch_size=kw.get("batch_size") or 16)

    class VectorStoreFactory:
        @staticmethod
        def create(cfg):
            store_calls.append({"backend": cfg.backend, "collection_name": cfg.collection_name,
                                "persist_directory": cfg.persist_directory, "distance_metric": cfg.distance_metric})
            return stores[cfg.collection_name]

    class ConfigLoader:
        @staticmethod
        def load_toolkit_config(name):
            raise FileNotFoundError(f"configs/rag/rag_tools/{name}.yaml")

    def mod(name, **attrs):
        m = types.ModuleType(name)
        m.__dict__.update(attrs)
        sys.modules[name] = m
        return m

    mod("utu.rag.embeddings.factory", EmbedderFactory=EmbedderFactory)
    mod("utu.rag.storage", VectorStoreFactory=VectorStoreFactory)
    mod("utu.config", ConfigLoader=ConfigLoader)
    mod("utu.utils").__path__ = []
    mod("utu.utils.log", get_logger=logging.getLogger)
    rag = sys.modules["utu.rag"]
    rag.Document, rag.Chunk, rag.VectorStoreConfig = base.Document, base.Chunk, config.VectorStoreConfig
    sys.modules["utu.rag.knowledge_builder"].RecursiveTextSplitter = mods["chunker"].RecursiveTextSplitter

    def load(name, rel):
        spec = importlib.util.spec_from_file_location(name, os.path.join(REF, rel))
        m = importlib.util.module_from_spec(spec)
        sys.modules[name] = m
        spec.loader.exec_module(m)
        return m

    KnowledgeBuilder = load("utu.rag.knowledge_builder.base_builder",
                            "utu/rag/knowledge_builder/base_builder.py").KnowledgeBuilder
    CourseSearcher = load("utu.rag.knowledge_retrieval.chroma_retrical_text2sql",
                          "utu/rag/knowledge_retrieval/chroma_retrical_text2sql.py").CourseSearcher

    docs_a, docs_b, docs_c = documents(3, 9, "a"), documents(4, 5, "b"), documents(5, 6, "c")
    kb_cfg = {"chunking": {"chunk_size": 300, "chunk_overlap": 30},
              "embedding": {"provider": "local", "base_url": "http://embed:8080", "batch_size": 16},
              "batch_delay": 0.0}
    store = Store(base.Chunk)
    stores["t2s_collection"] = store
    kb = KnowledgeBuilder(store, config.KnowledgeBuilderConfig(**kb_cfg))
    D = lambda ds: [base.Document(id=d["id"], content=d["content"], metadata=dict(d["metadata"])) for d in ds]  # noqa: E731
    steps = []
    for name, call in [("build_a", lambda: kb.build_from_documents(D(docs_a))),
                       ("add_b", lambda: kb.add_documents(D(docs_b)))]:
        st = asyncio.run(call())
        steps.append({"step": name, "status": status(st), "store_ids": list(store.ids)})
    snapshot = [{"id": i, "content": c, "metadata": m} for i, c, m in zip(store.ids, store.docs, store.metas)]

    os.environ["VECTOR_STORE_PATH"] = "/tmp/t2s_store"
    os.environ["UTU_EMBEDDING_URL"] = "http://embed:8080"
    cs = CourseSearcher(collection_name="t2s_collection")
    searches = []
    for q, k, fc in [("revenue by region", 5, None), ("course grade", 3, [{"title": "t1"}]),
                     ("student enrolment", 4, [{"page": {"$gte": 4}}, {"title": {"$in": ["t0", "t2"]}}]),
                     ("revenue by region", 2, [{"source": "b_2.md"}]), ("warehouse", 50, [{"year": 2021}])]:
        searches.append({"query": q, "top_k": k, "filter_conditions": fc,
                         "results": asyncio.run(cs.search(q, top_k=k, filter_conditions=fc))})
    cache_size = len(cs._embedding_cache)

    st = asyncio.run(kb.build_from_documents(D(docs_c), rebuild=True))
    steps.append({"step": "rebuild_c", "status": status(st), "store_ids": list(store.ids)})

    out = {"dim": HashEmbedder().dim, "kb_config": kb_cfg, "docs": {"a": docs_a, "b": docs_b, "c": docs_c},
           "steps": steps, "store_after_add_b": snapshot, "embedder_factory_calls": emb_calls,
           "store_factory_calls": store_calls, "course_searches": searches, "embedding_cache_size": cache_size,
           "env": {"VECTOR_STORE_PATH": "/tmp/t2s_store", "UTU_EMBEDDING_URL": "http://embed:8080"}}
    with open(os.path.join(HERE, "builder.json"), "w") as f:
        json.dump(out, f, indent=0, ensure_ascii=False)
    print("wrote", os.path.join(HERE, "builder.json"), len(snapshot), "chunks")


if __name__ == "__main__":
    main()

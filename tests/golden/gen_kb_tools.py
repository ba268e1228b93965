"""Golden fixtures for the KB-search tools from the REFERENCE's own code.

Runs only in the build container (reference tree read-only at /root/reference; no bytecode written).
The reference's KBSearchToolkit (utu/rag/rag_tools/kb_search_toolkit.py) and BaseRAGToolkit
(rag_tools/base_toolkit.py) are loaded from their source files and run as written:
``kb_embedding_search`` (:99-300), ``kb_file_search`` (:446-676), ``_build_metadata_filters``
(:63-96), ``_create_retriever`` + the per-collection store cache (base_toolkit.py:71-137), and the
reference ``VectorRetriever`` (base_retriever.py) they build.  Their imports that need packages
absent here (openai-agents, mcp, sqlmodel / SQLAlchemy, chromadb) are provided as small modules
registered in sys.modules before loading -- each one stands in for a plug-in point or plumbing
outside the hot path, never for code under test:
  utu.config.ToolkitConfig        a holder of the toolkit's ``config`` dict (agent_config.py:17)
  utu.tools.base                  AsyncBaseToolkit (stores the config) + register_tool (identity)
  utu.rag.api.database            the SQLite KnowledgeBase table -> a dict kb_id -> collection
  utu.rag.storage                 VectorStoreFactory -> the FAISS-semantics oracle store with
                                  Chroma's add / where / metadata conventions (chroma_store.py:64-148)
  utu.rag.embeddings.factory      EmbedderFactory -> a table embedder (query -> fixed vector)
  utu.rag.rerankers.factory       RerankerFactory -> raises (the HTTP reranker is unreachable
                                  offline; the tools' own no-reranker / rerank-failure paths run)
Output: kb_tools.json (inputs: the KB rows, the queries' vectors; expected: the tools' JSON strings,
the RetrieverConfig _create_retriever builds, the store-factory calls).
"""
from __future__ import annotations

import asyncio
import importlib.util
import json
import os
import sys
import types

sys.dont_write_bytecode = True
REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.path.insert(0, HERE)

import numpy as np  # noqa: E402

from oracle import ref_numpy as R  # noqa: E402
from gen_golden import load_reference  # noqa: E402

DIM = 64


def kb_rows():
    """Documents with content chunks + one summary vector each (processors.py:387-407, :423-464)."""
    rows = []
    vec_seed = 0
    for kb in (1, 2):
        for d in range(24 if kb == 1 else 6):
            doc = f"kb{kb}_doc{d}"
            meta = {"source": f"file_{d}.pdf", "author": f"a{d % 3}", "year": 2019 + d % 5,
                    "summary": f"summary of document {d} about topic {d % 4}"}
            for i in range(5):
                rows.append({"kb": kb, "id": f"{doc}_chunk_{i}", "document_id": doc, "content": f"content {d}.{i}",
                             "chunk_index": i, "metadata": {**meta, "index_type": "index_content"}, "vec": vec_seed})
                vec_seed += 1
            rows.append({"kb": kb, "id": f"{doc}_summary", "document_id": doc,
                         "content": f"file_{d}.pdf\n{meta['summary']}", "chunk_index": -1,
                         "metadata": {**meta, "index_type": "index_summary", "_derived_files_etags": "e"},
                         "vec": vec_seed})
            vec_seed += 1
    return rows


def vectors(n):
    return R.gen_rows(41, 0, n, DIM)


def _match(meta, where):
    """Chroma where-clause semantics on one metadata dict (chroma_store.py:104-116)."""
    for key, cond in where.items():
        if key == "$and":
            if not all(_match(meta, c) for c in cond):
                return False
            continue
        if key == "$or":
            if not any(_match(meta, c) for c in cond):
                return False
            continue
        if not (isinstance(cond, dict) and cond and all(k.startswith("$") for k in cond)):
            cond = {"$eq": cond}
        if key not in meta:
            return False
        v = meta[key]
        for op, x in cond.items():
            ok = {"$eq": lambda: v == x, "$ne": lambda: v != x, "$in": lambda: v in x, "$nin": lambda: v not in x,
                  "$gt": lambda: v > x, "$gte": lambda: v >= x, "$lt": lambda: v < x, "$lte": lambda: v <= x}[op]()
            if not ok:
                return False
    return True


class ChromaLikeOracleStore:
    """add_chunks / search with Chroma's conventions (stored metadata = {document_id, chunk_index,
    **non-None chunk metadata}; where = pre-filter) and FAISS's exact cosine arithmetic (oracle)."""

    def __init__(self, Chunk):
        self.Chunk = Chunk
        self.ids, self.docs, self.metas, self.vecs = [], [], [], []

    async def add_chunks(self, chunks):
        for c in chunks:
            self.ids.append(c.id)
            self.docs.append(c.content)
            self.metas.append({"document_id": c.document_id, "chunk_index": c.chunk_index,
                               **{k: v for k, v in (c.metadata or {}).items() if v is not None}})
            self.vecs.append(np.asarray(c.embedding, np.float32))

    async def search(self, query_embedding, top_k=5, filters=None):
        stored = R.process_rows(np.stack(self.vecs), "cosine", "f32")
        q = R.process_queries(np.asarray([query_embedding], np.float32), "cosine")
        allowed = np.array([_match(m, filters) for m in self.metas]) if filters else None
        s, r = R.search(stored, "f32", q, min(top_k, len(self.ids)), allowed)
        out = []
        for sc, row in zip(s[0], r[0]):
            if row < 0:
                continue
            m = dict(self.metas[row])
            out.append((self.Chunk(id=self.ids[row], document_id=m.get("document_id", ""), content=self.docs[row],
                                   chunk_index=m.get("chunk_index", 0), metadata=m),
                        float(np.float32(sc))))  # the store reports fp32 similarities
        return out


def load_toolkit(mods, stores, kb_table, factory_calls):
    def mod(name, **attrs):
        m = types.ModuleType(name)
        m.__dict__.update(attrs)
        sys.modules[name] = m
        return m

    class ToolkitConfig:
        def __init__(self, config=None, name=None, **kw):
            self.config = config or {}
            self.name = name
            self.activated_tools = None

    class AsyncBaseToolkit:
        def __init__(self, config=None):
            if not isinstance(config, ToolkitConfig):
                config = ToolkitConfig(config=config or {}, name=type(self).__name__)
            self.config = config

    def register_tool(fn=None, **kw):
        return fn if fn is not None else (lambda f: f)

    class _Col:
        def __eq__(self, other):
            return ("id", other)

    class KnowledgeBase:
        id = _Col()

    class _Query:
        def __init__(self):
            self.kb_id = None

        def filter(self, cond):
            self.kb_id = cond[1]
            return self

        def first(self):
            e = kb_table.get(self.kb_id)
            return None if e is None else types.SimpleNamespace(id=self.kb_id, name=e[1], collection_name=e[0])

    class _Session:
        def query(self, _model):
            return _Query()

        def close(self):
            pass

    def get_db():
        yield _Session()

    class VectorStoreFactory:
        @staticmethod
        def create(config):
            factory_calls.append({"backend": config.backend, "persist_directory": config.persist_directory,
                                  "collection_name": config.collection_name,
                                  "distance_metric": config.distance_metric})
            return stores[config.collection_name]

    class EmbedderFactory:
        @staticmethod
        def create(backend="auto", **kw):
            raise RuntimeError("embedder is injected")

    class RerankerFactory:
        @staticmethod
        def create(backend="auto", **kw):
            raise RuntimeError(f"reranker backend {backend!r} unreachable offline")

    mod("utu.config", ToolkitConfig=ToolkitConfig)
    tools_pkg = mod("utu.tools")
    tools_pkg.__path__ = []
    mod("utu.tools.base", AsyncBaseToolkit=AsyncBaseToolkit, register_tool=register_tool)
    api = mod("utu.rag.api")
    api.__path__ = []
    mod("utu.rag.api.database", get_db=get_db, KnowledgeBase=KnowledgeBase)
    mod("utu.rag.storage", VectorStoreFactory=VectorStoreFactory)
    mod("utu.rag.embeddings.factory", EmbedderFactory=EmbedderFactory)
    mod("utu.rag.rerankers.factory", RerankerFactory=RerankerFactory)
    kr = sys.modules["utu.rag.knowledge_retrieval"]
    kr.VectorRetriever = mods["retriever"].VectorRetriever
    pkg = mod("utu.rag.rag_tools")
    pkg.__path__ = [os.path.join(REF, "utu/rag/rag_tools")]
    for name in ("base_toolkit", "kb_search_toolkit"):
        spec = importlib.util.spec_from_file_location(f"utu.rag.rag_tools.{name}",
                                                      os.path.join(REF, f"utu/rag/rag_tools/{name}.py"))
        m = importlib.util.module_from_spec(spec)
        sys.modules[spec.name] = m
        spec.loader.exec_module(m)
    return sys.modules["utu.rag.rag_tools.kb_search_toolkit"].KBSearchToolkit


class TableEmbedder:
    def __init__(self, table):
        self.table = table

    async def embed_query(self, q):
        return self.table[q].tolist()


CASES = [
    # (tool, kwargs)
    ("kb_embedding_search", {"kb_id": 1, "query": "q0"}),
    ("kb_embedding_search", {"kb_id": 1, "query": "q1", "top_k": 5, "metadata_filters": {"source": "file_3.pdf"}}),
    ("kb_embedding_search", {"kb_id": 1, "query": "q2", "top_k": 4,
                             "metadata_filters": {"source": {"$in": ["file_1.pdf", "file_7.pdf", "file_9.pdf"]},
                                                  "year": {"$gte": 2021}}}),
    ("kb_embedding_search", {"kb_id": 1, "query": "q3", "top_k": 6, "auto_rerank": False,
                             "metadata_filters": {"index_type": "index_content", "author": "a1"}}),
    ("kb_embedding_search", {"kb_id": 2, "query": "q4", "top_k": 3}),
    ("kb_embedding_search", {"kb_id": 99, "query": "q0"}),
    ("kb_file_search", {"kb_id": 1, "query": "q5"}),
    ("kb_file_search", {"kb_id": 1, "query": "q6", "top_k": 5, "auto_rerank": False, "include_summary": False}),
    ("kb_file_search", {"kb_id": 1, "query": "q7", "top_k": 4, "metadata_filters": {"author": "a2"}}),
    ("kb_file_search", {"kb_id": 2, "query": "q8", "top_k": 10, "auto_rerank": False}),
    ("kb_file_search", {"kb_id": 1, "query": "q9", "top_k": 1}),
]
TOOLKIT_CONFIGS = [{}, {"top_k": 4, "recall_multiplier": 2,
                        "vector_store": {"persist_directory": "/tmp/kbstore", "distance_metric": "cosine"}}]


def main():
    mods = load_reference()
    Chunk = mods["base"].Chunk
    rows = kb_rows()
    vecs = vectors(len(rows))
    rng = np.random.default_rng(5)
    # queries near some rows (summary and content), plus noise
    picks = rng.choice(len(rows), 10, replace=False)
    qv = {f"q{i}": (vecs[p] / np.linalg.norm(vecs[p]) + 0.3 * rng.standard_normal(DIM) / np.sqrt(DIM)).astype(np.float32)
          for i, p in enumerate(picks)}
    kb_table = {1: ("kb_collection_1", "KB one"), 2: ("kb_collection_2", "KB two")}
    out = {"dim": DIM, "rows": [{k: v for k, v in r.items()} for r in rows], "vectors_seed": 41,
           "queries": {k: v.tolist() for k, v in qv.items()}, "kb_table": {str(k): v for k, v in kb_table.items()},
           "runs": []}
    for cfg in TOOLKIT_CONFIGS:
        stores = {}
        for kb, (coll, _) in kb_table.items():
            st = ChromaLikeOracleStore(Chunk)
            sel = [r for r in rows if r["kb"] == kb]
            asyncio.run(st.add_chunks([Chunk(id=r["id"], document_id=r["document_id"], content=r["content"],
                                             chunk_index=r["chunk_index"], metadata=dict(r["metadata"]),
                                             embedding=vecs[r["vec"]].tolist()) for r in sel]))
            stores[coll] = st
        calls = []
        KBSearchToolkit = load_toolkit(mods, stores, kb_table, calls)
        tk = KBSearchToolkit(config=cfg)
        tk._embedder_cache = TableEmbedder(qv)
        run = {"toolkit_config": cfg, "outputs": []}
        for tool, kw in CASES:
            run["outputs"].append({"tool": tool, "kwargs": kw, "json": asyncio.run(getattr(tk, tool)(**kw))})
        ret = asyncio.run(tk._create_retriever(1, 7))
        run["create_retriever"] = {"top_k": ret.config.top_k, "similarity_threshold": ret.config.similarity_threshold,
                                   "enable_reranking": ret.config.enable_reranking,
                                   "reranker": ret.reranker is not None}
        run["store_factory_calls"] = calls
        run["metadata_filters"] = [{"in": f, "out": tk._build_metadata_filters(f)} for f in
                                   [None, {}, {"source": "a.pdf"}, {"source": {"$in": ["a", "b"]}},
                                    {"a": 1, "b": {"$gte": 2}, "c": {"x": 1}}]]
        out["runs"].append(run)
    with open(os.path.join(HERE, "kb_tools.json"), "w") as f:
        json.dump(out, f, indent=0, ensure_ascii=False)
    print("wrote", os.path.join(HERE, "kb_tools.json"))


if __name__ == "__main__":
    main()

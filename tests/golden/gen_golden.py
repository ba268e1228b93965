"""Generate the golden fixtures under tests/golden/ by running the REFERENCE's own code.

Runs only in the build container, where the reference tree is mounted read-only
at /root/reference (it never travels to the GPU box; the fixtures do).  The
reference package root (utu/__init__.py) needs openai-agents, which is absent,
so the leaf modules are loaded with ``utu`` / ``utu.rag`` / ``utu.db``
pre-registered as bare namespace packages pointing into the tree.  No bytecode
is written into the reference (sys.dont_write_bytecode).

Fixtures produced (all small; inputs + expected outputs only):
  c1_retrieval.npz / .json  config C1 (1000x128 fp32 corpus, 16 queries, top-5)
        through reference VectorRetriever.batch_retrieve (base_retriever.py:82-99)
        at similarity_threshold 0.0 (the tool path, base_toolkit.py:126-130), the
        default 0.7 (config.py:46), and a metadata-filtered variant.
  ties.npz / .json       20k x 256 corpus with planted exact duplicates: the
        (score desc, row asc) tie order.
  chunker.json           RecursiveTextSplitter (chunker.py:10-121) at 500/50 and 1000/100.
  service_embedder.json  ServiceEmbedder.embed_texts/embed_query wire decode and
        batch split (service_embedder.py:73-177), transport monkeypatched in-process.
  corpus_sha256.json     SHA-256 of stored synthetic corpora (bf16/f16/f32), so the GPU
        box can rebuild them with the device generator and compare bytes.

The vector store plugged into the reference retriever is the oracle's restatement
of FAISSVectorStore cosine semantics (faiss itself is absent, see oracle/).
"""
from __future__ import annotations

import asyncio
import base64
import hashlib
import importlib
import json
import os
import sys
import types

sys.dont_write_bytecode = True
REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402

import oracle  # noqa: E402
from oracle import ref_numpy as R  # noqa: E402


def _bare_pkg(name: str, rel: str):
    m = types.ModuleType(name)
    m.__path__ = [os.path.join(REF, rel)]
    sys.modules[name] = m


def load_reference():
    for name, rel in [("utu", "utu"), ("utu.rag", "utu/rag"), ("utu.db", "utu/db"), ("utu.config", "utu/config"),
                      ("utu.rag.knowledge_builder", "utu/rag/knowledge_builder"),
                      ("utu.rag.embeddings", "utu/rag/embeddings"),
                      ("utu.rag.knowledge_retrieval", "utu/rag/knowledge_retrieval"),
                      ("utu.rag.rerankers", "utu/rag/rerankers")]:
        _bare_pkg(name, rel)
    mods = {}
    mods["base"] = importlib.import_module("utu.rag.base")
    mods["config"] = importlib.import_module("utu.rag.config")
    mods["retriever"] = importlib.import_module("utu.rag.knowledge_retrieval.base_retriever")
    mods["chunker"] = importlib.import_module("utu.rag.knowledge_builder.chunker")
    mods["service"] = importlib.import_module("utu.rag.embeddings.service_embedder")
    return mods


class OracleStore:
    """FAISSVectorStore cosine semantics restated (faiss_store.py:89-199) with Chroma
    pre-filter semantics for ``filters`` (chroma_store.py:104-120: exact top-k among
    matching rows).  Built on oracle.ref_numpy."""

    def __init__(self, Chunk, vectors: np.ndarray, metas: list[dict]):
        self.Chunk = Chunk
        self.stored = R.process_rows(vectors, "cosine", "f32")
        self.metas = metas

    async def search(self, query_embedding, top_k=5, filters=None):
        q = R.process_queries(np.asarray([query_embedding], np.float32), "cosine")
        allowed = None
        if filters:
            allowed = np.array([all(m.get(k) == v for k, v in filters.items()) for m in self.metas])
        s, r = R.search(self.stored, "f32", q, top_k, allowed)
        out = []
        for score, row in zip(s[0], r[0]):
            if row < 0:
                continue
            m = self.metas[row]
            out.append((self.Chunk(id=f"chunk_{row}", document_id=m["document_id"], content=f"text {row}",
                                   chunk_index=int(m["chunk_index"]), metadata=dict(m)), float(score)))
        return out


class TableEmbedder:
    def __init__(self, table: dict[str, np.ndarray]):
        self.table = table

    async def embed_query(self, query):
        return self.table[query].tolist()

    async def embed_texts(self, texts):
        return [self.table[t].tolist() for t in texts]


def _results_to_json(batch):
    return [[{"chunk_id": rr.chunk.id, "score": rr.score, "rank": rr.rank} for rr in res] for res in batch]


def gen_c1(mods):
    Chunk = mods["base"].Chunk
    RetrieverConfig = mods["config"].RetrieverConfig
    VectorRetriever = mods["retriever"].VectorRetriever
    n, dim = 1000, 128
    corpus = R.gen_rows(0, 0, n, dim)
    rng = np.random.default_rng(1)
    q = np.empty((16, dim), np.float32)
    planted = rng.choice(n, 16, replace=False)
    # half the queries are planted near a corpus row (scores > 0.7), half are random
    for i in range(16):
        noise = rng.standard_normal(dim).astype(np.float32)
        base = corpus[planted[i]] / np.linalg.norm(corpus[planted[i]])
        q[i] = base + (0.3 if i % 2 == 0 else 20.0) * noise / np.linalg.norm(noise)
    metas = [{"document_id": f"doc_{r // 10}", "chunk_index": r % 10, "group": f"g{r % 4}"} for r in range(n)]
    store = OracleStore(Chunk, corpus, metas)
    names = [f"query {i}" for i in range(16)]
    emb = TableEmbedder(dict(zip(names, q)))
    out = {}
    for tag, thr in [("thr0", 0.0), ("thr_default", None)]:
        cfg = RetrieverConfig(top_k=5, similarity_threshold=thr) if thr is not None else RetrieverConfig(top_k=5)
        ret = VectorRetriever(vector_store=store, embedder=emb, config=cfg)
        out[tag] = _results_to_json(asyncio.run(ret.batch_retrieve(names, top_k=5)))
    ret = VectorRetriever(vector_store=store, embedder=emb, config=RetrieverConfig(top_k=5, similarity_threshold=0.0))
    out["filtered_g1"] = _results_to_json(asyncio.run(ret.batch_retrieve(names, top_k=5, filters={"group": "g1"})))
    np.savez_compressed(os.path.join(HERE, "c1_retrieval.npz"), corpus=corpus, queries=q)
    with open(os.path.join(HERE, "c1_retrieval.json"), "w") as f:
        json.dump({"config": "C1: 1000x128 fp32 corpus (oracle generator seed 0), 16 queries, top-5, cosine",
                   "metas": metas, "query_names": names, "results": out}, f, indent=0)


def gen_ties(mods):
    Chunk = mods["base"].Chunk
    RetrieverConfig = mods["config"].RetrieverConfig
    VectorRetriever = mods["retriever"].VectorRetriever
    n, dim = 20000, 256
    corpus = R.gen_rows(7, 0, n, dim)
    rng = np.random.default_rng(7)
    src = rng.choice(n, 12, replace=False)
    dups = {}
    for s in src:  # 3 exact copies of each source row at random later positions
        dst = rng.choice(n, 3, replace=False)
        corpus[dst] = corpus[s]
        dups[int(s)] = [int(d) for d in dst]
    q = np.stack([corpus[s] for s in src[:8]] +
                 [corpus[s] * 2.0 + rng.standard_normal(dim).astype(np.float32) * 500 for s in src[8:]]).astype(np.float32)
    metas = [{"document_id": f"doc_{r // 50}", "chunk_index": r % 50} for r in range(n)]
    store = OracleStore(Chunk, corpus, metas)
    names = [f"tie query {i}" for i in range(len(q))]
    emb = TableEmbedder(dict(zip(names, q)))
    ret = VectorRetriever(vector_store=store, embedder=emb, config=RetrieverConfig(top_k=10, similarity_threshold=0.0))
    res = _results_to_json(asyncio.run(ret.batch_retrieve(names, top_k=10)))
    np.savez_compressed(os.path.join(HERE, "ties.npz"), queries=q,
                        dup_src=np.array(list(dups.keys()), np.int64),
                        dup_dst=np.array(list(dups.values()), np.int64))
    with open(os.path.join(HERE, "ties.json"), "w") as f:
        json.dump({"config": "20000x256 fp32 corpus (oracle generator seed 7) with corpus[dup_dst[i]] = corpus[dup_src[i]]",
                   "results": res}, f, indent=0)


def _word_text(rng, n_words):
    words = ["alpha", "beta", "gamma", "delta", "retrieval", "vector", "chunk", "embedding", "GPU", "kernel",
             "x", "knowledge", "base", "search", "MI355X"]
    out = []
    for i in range(n_words):
        w = words[rng.integers(len(words))]
        r = rng.random()
        out.append(w + (".\n\n" if r < 0.03 else ".\n" if r < 0.06 else ". " if r < 0.12 else " "))
    return "".join(out)


def gen_chunker(mods):
    RecursiveTextSplitter = mods["chunker"].RecursiveTextSplitter
    ChunkingConfig = mods["config"].ChunkingConfig
    rng = np.random.default_rng(3)
    texts = [_word_text(rng, n) for n in (5, 80, 400, 1500)]
    texts.append("hello world." * 120)
    texts.append("z" * 2500)
    texts.append("")
    cases = []
    for size, overlap in [(500, 50), (1000, 100), (300, 0)]:
        sp = RecursiveTextSplitter(ChunkingConfig(chunk_size=size, chunk_overlap=overlap))
        cases.append({"chunk_size": size, "chunk_overlap": overlap,
                      "chunks": [sp.split_text(t) for t in texts]})
    with open(os.path.join(HERE, "chunker.json"), "w") as f:
        json.dump({"texts": texts, "cases": cases}, f)


def gen_service_embedder(mods):
    svc = mods["service"]
    dim = 24
    calls = []

    def fake_request(url, json_data, **kw):
        calls.append({"url": url.rsplit("/", 1)[-1], "n": len(json_data.get("docs", [json_data.get("query")]))})
        if "docs" in json_data:
            arr = np.stack([R.gen_rows(11, hash_text(t), 1, dim)[0] / 1e5 for t in json_data["docs"]]).astype(np.float32)
        else:
            arr = (R.gen_rows(11, hash_text(json_data["query"]), 1, dim)[0] / 1e5).astype(np.float32)
        return {"embedding": base64.b64encode(arr.tobytes()).decode("ascii"), "shape": list(arr.shape)}

    def hash_text(t):
        return int(hashlib.sha256(t.encode()).hexdigest()[:8], 16) % 100000

    class _Resp:
        def raise_for_status(self):
            pass

        def json(self):
            return "fake-model"

    svc.make_request_with_retry = fake_request
    svc.requests = types.SimpleNamespace(get=lambda *a, **k: _Resp(), exceptions=svc.requests.exceptions)
    emb = svc.ServiceEmbedder(service_url="http://embed.invalid:8081/", batch_size=50)
    texts = [f"passage number {i}" for i in range(120)]
    vecs = asyncio.run(emb.embed_texts(texts))
    qv = asyncio.run(emb.embed_query("what is the chunk size?"))
    with open(os.path.join(HERE, "service_embedder.json"), "w") as f:
        json.dump({"texts": texts, "batch_size": 50, "calls": calls, "embeddings": vecs, "query": "what is the chunk size?",
                   "query_embedding": qv, "dim": dim,
                   "generator": "row = oracle gen_rows(seed=11, row=int(sha256(text)[:8],16)%100000, dim=24)/1e5"}, f)


def gen_sha():
    out = {}
    for dim, n in [(128, 1000), (768, 4096), (1024, 4096)]:
        for dtype in ["bf16", "f16", "f32"]:
            st = oracle.c_build_synthetic(0, 0, n, dim, dtype, "cosine", 4)
            out[f"seed0_rows{n}_dim{dim}_{dtype}_cosine"] = hashlib.sha256(st.tobytes()).hexdigest()
    st = oracle.c_build_synthetic(0, 0, 1000, 128, "bf16", "ip", 4)
    out["seed0_rows1000_dim128_bf16_ip"] = hashlib.sha256(st.tobytes()).hexdigest()
    with open(os.path.join(HERE, "corpus_sha256.json"), "w") as f:
        json.dump(out, f, indent=1)


def main():
    mods = load_reference()
    gen_c1(mods)
    gen_ties(mods)
    gen_chunker(mods)
    gen_service_embedder(mods)
    gen_sha()
    print("golden fixtures written to", HERE)


if __name__ == "__main__":
    main()

"""The other two callers on either side of the search path: KnowledgeBuilder (ingest) and CourseSearcher
(text2sql schema retrieval).

KnowledgeBuilder restates utu/rag/knowledge_builder/base_builder.py:17-182:
  * the embedder comes from the config (:37-53): provider "local" -> the embedding service,
    "openai" -> the OpenAI-compatible client, and here also "rocm" / "huggingface" -> the in-process
    TorchRocmEmbedder; an ``embedder=`` argument overrides (the reference has no injection point);
  * build_from_documents (:58-118): under one asyncio lock, status "running" with total_documents;
    ``rebuild`` clears the store first; each document is split (RecursiveTextSplitter, :148) and
    embedded; a document that fails is recorded in ``errors`` as ``"Error processing document {id}:
    {e}"`` and skipped; ALL chunks then go to the store in ONE add_chunks call (:100-102); status
    "completed" with end_time, or "failed" (error appended) and the exception re-raised;
  * chunk i of document d: id = md5(f"{d}_{i}").hexdigest() (:171-182), document_id d, chunk_index i,
    metadata = {**document.metadata, "chunk_index": i, "total_chunks": n} (:152-166).
What changes: the embedder runs over full batches that span documents (the reference embeds one
document at a time, :150), and with the in-process embedder and a HipVectorStore the vectors stay on
the GPU (embed_texts_device -> add_chunks_device).  If a packed batch fails, its documents are embedded
one by one so the failure is attributed to the document that caused it, as in the reference.

CourseSearcher restates utu/rag/knowledge_retrieval/chroma_retrical_text2sql.py:45-196:
  * config (:83-110): a dict with "embedding" and "vector_store" sections (the reference loads it from
    configs/rag/rag_tools/<config_name>.yaml; here it is passed in, or read from that file when present,
    else the reference's environment defaults); ``vector_save_path`` overrides persist_directory (:67-68);
  * the store is VectorStoreFactory.create(VectorStoreConfig(backend, collection_name,
    persist_directory, distance_metric)) (:70-77), the embedder EmbedderFactory.create(backend, ...)
    with the reference's parameter mapping (:112-142; an unknown backend falls back to "service");
  * search (:148-196): per-query embedding cache, ``filter_conditions`` -> the single condition or
    {"$and": [...]}, store.search(query_embedding=..., top_k, filters), one dict per hit with chunk_id,
    document_id, content, chunk_index, metadata, score.
Added: ``search_batch`` embeds the uncached queries in one embedder batch and answers all queries with
one index launch (HipVectorStore.search_batch).
"""
from __future__ import annotations

import asyncio
import hashlib
import logging
import os
from datetime import datetime
from typing import Any

from .base import BaseKnowledgeBuilder, BaseVectorStore, BuildStatus, Chunk, Document
from .chunker import RecursiveTextSplitter
from .config import KnowledgeBuilderConfig, VectorStoreConfig
from .embeddings import EmbedderFactory

logger = logging.getLogger(__name__)


def chunk_id(document_id: str, chunk_index: int) -> str:
    """base_builder.py:171-182."""
    return hashlib.md5(f"{document_id}_{chunk_index}".encode()).hexdigest()


def _builder_embedder(config: KnowledgeBuilderConfig):
    """base_builder.py:37-53, plus the in-process providers."""
    emb = config.embedding
    if emb.provider == "local":
        return EmbedderFactory.create(backend="service", service_url=emb.base_url, batch_size=emb.batch_size,
                                      batch_delay=config.batch_delay)
    if emb.provider in ("rocm", "huggingface"):
        return EmbedderFactory.create(backend="rocm", model_name_or_path=emb.model, batch_size=emb.batch_size)
    return EmbedderFactory.create(backend="openai", model=emb.model, api_key=emb.api_key, base_url=emb.base_url,
                                  batch_size=emb.batch_size, batch_delay=config.batch_delay)


class KnowledgeBuilder(BaseKnowledgeBuilder):
    def __init__(self, vector_store: BaseVectorStore, config: KnowledgeBuilderConfig | None = None,
                 embedder=None, embed_batch: int | None = None):
        self.vector_store = vector_store
        self.config = config or KnowledgeBuilderConfig()
        self.text_splitter = RecursiveTextSplitter(config=self.config.chunking)
        self.embedder = embedder if embedder is not None else _builder_embedder(self.config)
        self.embed_batch = int(embed_batch or getattr(self.embedder, "batch_size", 64) or 64)
        self._device = hasattr(self.embedder, "embed_texts_device") and hasattr(vector_store, "add_chunks_device")
        self._build_status = BuildStatus(status="idle")
        self._lock = asyncio.Lock()

    async def build_from_documents(self, documents: list[Document], rebuild: bool = False) -> BuildStatus:
        async with self._lock:
            st = BuildStatus(status="running", total_documents=len(documents), processed_documents=0,
                             total_chunks=0, start_time=datetime.now().isoformat())
            self._build_status = st
            try:
                if rebuild:
                    logger.info("Clearing existing knowledge base...")
                    await self.vector_store.clear()
                chunks, embs = await self._process_all(documents, st)
                if chunks:
                    logger.info("Adding %d chunks to vector store...", len(chunks))
                    await self._add(chunks, embs)
                st.status = "completed"
                st.end_time = datetime.now().isoformat()
            except Exception as e:
                st.status = "failed"
                st.errors.append(str(e))
                st.end_time = datetime.now().isoformat()
                logger.error("Knowledge base build failed: %s", e)
                raise
            return st

    async def add_documents(self, documents: list[Document]) -> BuildStatus:
        return await self.build_from_documents(documents, rebuild=False)

    async def get_build_status(self) -> BuildStatus:
        return self._build_status

    # ------------------------------------------------------------------ internals
    def _split(self, document: Document) -> list[Chunk]:
        texts = self.text_splitter.split_text(document.content, document.metadata)
        return [Chunk(id=chunk_id(document.id, i), document_id=document.id, content=t, chunk_index=i,
                      metadata={**(document.metadata or {}), "chunk_index": i, "total_chunks": len(texts)})
                for i, t in enumerate(texts)]

    async def _embed(self, texts: list[str]):
        if self._device:
            return self.embedder.embed_texts_device(texts)
        return await self.embedder.embed_texts(texts)

    async def _process_all(self, documents: list[Document], st: BuildStatus):
        """Split every document, embed in batches spanning documents, keep the reference's per-document
        success / error accounting.  Returns (chunks, embeddings in chunk order)."""
        ok_chunks: list[Chunk] = []
        ok_embs: list = []
        pending: list[tuple[int, Document, list[Chunk]]] = []  # (position, document, chunks)
        n_pending = 0

        def fail(doc: Document, e: Exception):
            msg = f"Error processing document {doc.id}: {e}"
            logger.error(msg)
            st.errors.append(msg)

        async def settle(entries):
            try:
                texts = [c.content for _, _, cs in entries for c in cs]
                embs = await self._embed(texts) if texts else []
            except Exception as e:
                if len(entries) == 1:
                    fail(entries[0][1], e)
                else:  # attribute the failure: one document at a time
                    for entry in entries:
                        await settle([entry])
                return
            o = 0
            for pos, doc, cs in entries:
                ok_chunks.extend(cs)
                ok_embs.append(embs[o:o + len(cs)])
                o += len(cs)
                # position of the last successful document, as the reference counts (base_builder.py:89)
                st.processed_documents = pos + 1
                st.total_chunks = len(ok_chunks)
                logger.info("Processed document %d/%d: %s, generated %d chunks", pos + 1, len(documents), doc.id,
                            len(cs))

        for pos, doc in enumerate(documents):
            try:
                cs = self._split(doc)
            except Exception as e:
                fail(doc, e)
                continue
            pending.append((pos, doc, cs))
            n_pending += len(cs)
            if n_pending >= self.embed_batch:
                await settle(pending)
                pending, n_pending = [], 0
        if pending:
            await settle(pending)
        return ok_chunks, ok_embs

    async def _add(self, chunks: list[Chunk], embs: list):
        if self._device:
            import torch

            parts = [e for e in embs if len(e)]
            self.vector_store.add_chunks_device(chunks, torch.cat(parts) if len(parts) > 1 else parts[0])
            return
        flat = [v for e in embs for v in e]
        for c, v in zip(chunks, flat):
            c.embedding = v
        await self.vector_store.add_chunks(chunks)


# ---------------------------------------------------------------------------------------------- text2sql
def _env_defaults() -> dict:
    """chroma_retrical_text2sql.py:97-110."""
    return {"embedding": {"backend": "service", "base_url": os.getenv("UTU_EMBEDDING_URL"), "batch_size": 16},
            "vector_store": {"backend": "chroma", "persist_directory": os.getenv("VECTOR_STORE_PATH"),
                             "distance_metric": "cosine"}}


def _load_toolkit_yaml(config_name: str) -> dict:
    """configs/rag/rag_tools/<name>.yaml under HIPRAG_CONFIG_DIR (default ./configs), ${oc.env:VAR[,default]}
    references resolved from the environment; the file's ``config`` section, as ToolkitConfig.config."""
    import re

    import yaml

    root = os.environ.get("HIPRAG_CONFIG_DIR", "configs")
    path = os.path.join(root, "rag", "rag_tools", f"{config_name}.yaml")
    with open(path, encoding="utf-8") as f:
        text = f.read()

    def env(m):
        name, _, default = m.group(1).partition(",")
        return os.environ.get(name.strip(), default.strip())

    data = yaml.safe_load(re.sub(r"\$\{oc\.env:([^}]*)\}", env, text)) or {}
    return dict(data.get("config", data))


class CourseSearcher:
    def __init__(self, collection_name: str = "demo_knowledge_base", vector_save_path: str | None = None,
                 config_name: str = "text2sql_retrieval", *, config: dict | None = None, vector_store=None,
                 embedder=None):
        self.config = config if config is not None else self._load_config(config_name)
        vs = dict(self.config.get("vector_store", {}))
        if vector_save_path:
            vs["persist_directory"] = vector_save_path
        if vector_store is None:
            from .storage import VectorStoreFactory

            vector_store = VectorStoreFactory.create(VectorStoreConfig(
                backend=vs.get("backend", "chroma"), collection_name=collection_name,
                persist_directory=vs.get("persist_directory") or VectorStoreConfig().persist_directory,
                distance_metric=vs.get("distance_metric", "cosine"), index_params=vs.get("index_params") or {}))
        self.vector_store = vector_store
        self.embedder = embedder if embedder is not None else self._init_embedder()
        self._embedding_cache: dict[str, list[float]] = {}

    @staticmethod
    def _load_config(config_name: str) -> dict:
        try:
            return _load_toolkit_yaml(config_name)
        except Exception as e:
            logger.warning("Failed to load config '%s.yaml': %s, using env defaults", config_name, e)
            return _env_defaults()

    def _init_embedder(self):
        ec = self.config.get("embedding", {})
        backend = ec.get("backend", "service")
        if backend == "service":
            params = {"service_url": ec.get("base_url"), "batch_size": ec.get("batch_size", 16)}
        elif backend == "openai":
            params = {"model": ec.get("model"), "api_key": ec.get("api_key"), "base_url": ec.get("base_url"),
                      "batch_size": ec.get("batch_size", 16)}
        elif backend in ("rocm", "huggingface", "local"):
            params = {k: v for k, v in ec.items() if k not in ("backend", "base_url", "api_key")}
            if "model" in params:
                params["model_name_or_path"] = params.pop("model")
        else:
            logger.warning("Unknown embedding backend '%s', using service as fallback", backend)
            backend, params = "service", {"service_url": os.getenv("UTU_EMBEDDING_URL"), "batch_size": 16}
        return EmbedderFactory.create(backend=backend, **params)

    def clear_embedding_cache(self):
        self._embedding_cache.clear()

    @staticmethod
    def _where(filter_conditions):
        if not filter_conditions:
            return None
        return filter_conditions[0] if len(filter_conditions) == 1 else {"$and": filter_conditions}

    @staticmethod
    def _rows(results) -> list[dict[str, Any]]:
        return [{"chunk_id": c.id, "document_id": c.document_id, "content": c.content, "chunk_index": c.chunk_index,
                 "metadata": c.metadata, "score": s} for c, s in results]

    async def search(self, query: str, top_k: int = 5, filter_conditions: list[dict[str, Any]] | None = None
                     ) -> list[dict[str, Any]]:
        if query in self._embedding_cache:
            q = self._embedding_cache[query]
        else:
            q = await self.embedder.embed_query(query)
            self._embedding_cache[query] = q
        results = await self.vector_store.search(query_embedding=q, top_k=top_k,
                                                 filters=self._where(filter_conditions))
        return self._rows(results)

    async def search_batch(self, queries: list[str], top_k: int = 5,
                           filter_conditions: list[dict[str, Any]] | None = None) -> list[list[dict[str, Any]]]:
        """``search`` for many queries: one embedder batch for the uncached ones, one index launch."""
        todo = list(dict.fromkeys(q for q in queries if q not in self._embedding_cache))
        if todo:
            embed_queries = getattr(self.embedder, "embed_queries", None)
            vecs = (await embed_queries(todo) if embed_queries is not None
                    else [await self.embedder.embed_query(q) for q in todo])
            for q, v in zip(todo, vecs):
                self._embedding_cache[q] = list(v)
        where = self._where(filter_conditions)
        if hasattr(self.vector_store, "search_batch"):
            res = self.vector_store.search_batch([self._embedding_cache[q] for q in queries], top_k, where)
        else:
            res = [await self.vector_store.search(query_embedding=self._embedding_cache[q], top_k=top_k,
                                                  filters=where) for q in queries]
        return [self._rows(r) for r in res]

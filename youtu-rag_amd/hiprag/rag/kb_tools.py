"""The KB-search tools over the MI355X store: mirror of the reference's agent-facing callers.

``BaseRAGToolkit`` restates utu/rag/rag_tools/base_toolkit.py:17-137 and ``KBSearchToolkit``
restates kb_search_toolkit.py:17-676 (``kb_embedding_search`` :99-300, ``kb_rerank`` :301-444,
``kb_file_search`` :446-676, ``_build_metadata_filters`` :63-96) with the same arguments, JSON
output (keys, order, ``round(score, 4)``, ``ensure_ascii=False, indent=2``), defaults and failure
behaviour; tests/golden/kb_tools.json (produced by running the reference toolkit itself,
tests/golden/gen_kb_tools.py) pins them.  What changes is only what sits under them:
  * stores come from hiprag's VectorStoreFactory (HipVectorStore: exact GPU search, where-clauses
    compiled to cached row bitmaps), cached per collection exactly as base_toolkit.py:79-91 does;
  * the embedder is hiprag's EmbedderFactory (in-process ``rocm`` embedder, or the reference's
    HTTP ``service`` wire format), cached once per toolkit (:71-77);
  * the reranker is the in-process cross-encoder when the config names ``rocm``; the reference's
    HTTP rerankers are unreachable here, which takes the tools' own no-reranker paths, as offline;
  * the KB id -> collection lookup (a SQLite ``KnowledgeBase`` query in the reference, :42-51, part of
    the FastAPI backend, outside the hot path) is ``config["kb_collections"]`` or an injected
    ``kb_resolver(kb_id) -> (collection_name, kb_name)``.
Reference quirks kept: ``file_search_top_k`` reads the same "top_k" key as content search (:34-35);
``kb_rerank`` passes ``top_n=`` to ``rerank()`` (:391-393), which the rerankers do not accept, so the
tool answers with its error JSON; an unknown kb_id fails before the not-found check (:46) with the
same error shape.
"""
from __future__ import annotations

import json
import logging
from typing import Any, Optional

from .base import Chunk, RetrievalResult
from .config import RetrieverConfig, VectorStoreConfig
from .retriever import VectorRetriever

logger = logging.getLogger(__name__)


class _ToolkitConfig:
    def __init__(self, config: dict | None = None, name: str | None = None):
        self.config = dict(config or {})
        self.name = name


class BaseRAGToolkit:
    """Shared store / embedder / retriever plumbing of the KB tools (base_toolkit.py:17-137)."""

    def __init__(self, config=None, *, kb_resolver=None, store_factory=None, embedder_factory=None):
        if not hasattr(config, "config"):
            config = _ToolkitConfig(config, type(self).__name__)
        self.config = config
        self.embedding_config = self.config.config.get("embedding", {})
        self.vector_store_base_config = self.config.config.get("vector_store", {})
        self._kb_resolver = kb_resolver
        self._store_factory = store_factory
        self._embedder_factory = embedder_factory
        self._embedder_cache = None
        self._vector_store_cache: dict[str, Any] = {}

    async def _get_kb_collection_name(self, kb_id: int) -> tuple[str, str]:
        if self._kb_resolver is not None:
            found = self._kb_resolver(kb_id)
        else:
            table = {str(k): v for k, v in (self.config.config.get("kb_collections") or {}).items()}
            v = table.get(str(kb_id))
            found = None if v is None else ((v, str(v)) if isinstance(v, str) else tuple(v))
        if found is None:  # the reference dereferences the missing row first (base_toolkit.py:45-46)
            raise AttributeError("'NoneType' object has no attribute 'name'")
        return found[0], found[1]

    def _build_embedder_params(self, embedding_config: Optional[dict] = None) -> dict:
        config = embedding_config or self.embedding_config
        backend = config.get("backend", "openai")
        if backend == "service":
            return {"service_url": config.get("base_url"), "batch_size": config.get("batch_size", 16)}
        return {"model": config.get("model"), "api_key": config.get("api_key"), "base_url": config.get("base_url"),
                "batch_size": config.get("batch_size", 16)}

    def _get_or_create_embedder(self):
        if self._embedder_cache is None:
            backend = self.embedding_config.get("backend", "openai")
            if self._embedder_factory is not None:
                create = self._embedder_factory
            else:
                from .embeddings import EmbedderFactory

                create = EmbedderFactory.create
            self._embedder_cache = create(backend=backend, **self._build_embedder_params())
        return self._embedder_cache

    def _get_or_create_vector_store(self, collection_name: str, persist_directory: str):
        if collection_name not in self._vector_store_cache:
            vs = self.vector_store_base_config
            cfg = VectorStoreConfig(backend=vs.get("backend", "chroma"), persist_directory=persist_directory,
                                    collection_name=collection_name,
                                    distance_metric=vs.get("distance_metric", "cosine"),
                                    index_params=vs.get("index_params") or {})
            if self._store_factory is not None:
                self._vector_store_cache[collection_name] = self._store_factory(cfg)
            else:
                from .storage import VectorStoreFactory

                self._vector_store_cache[collection_name] = VectorStoreFactory.create(cfg)
        return self._vector_store_cache[collection_name]

    async def _create_retriever(self, kb_id: int, top_k: int, embedder=None, persist_directory: Optional[str] = None,
                                similarity_threshold: float = 0.0) -> VectorRetriever:
        collection_name, _kb_name = await self._get_kb_collection_name(kb_id)
        persist_dir = persist_directory or self.vector_store_base_config.get("persist_directory",
                                                                             "./rag_data/vector_store")
        store = self._get_or_create_vector_store(collection_name, persist_dir)
        if embedder is None:
            embedder = self._get_or_create_embedder()
        cfg = RetrieverConfig(top_k=top_k, similarity_threshold=similarity_threshold, enable_reranking=False)
        return VectorRetriever(vector_store=store, embedder=embedder, config=cfg)


def _reranker_from(backend: str):
    from .rerankers import RerankerFactory

    return RerankerFactory.create(backend=backend)


class KBSearchToolkit(BaseRAGToolkit):
    """kb_embedding_search / kb_file_search / kb_rerank (kb_search_toolkit.py:17-676)."""

    def __init__(self, config=None, **kw):
        super().__init__(config, **kw)
        c = self.config.config
        self.default_top_k = c.get("top_k", 3)
        self.file_search_top_k = c.get("top_k", 15)
        self.recall_multiplier = c.get("recall_multiplier", 3)
        self.reranker_config = c.get("reranker", {})
        self.reranker = self._init_reranker()

    def _init_reranker(self):
        try:
            return _reranker_from(self.reranker_config.get("backend", "jina"))
        except Exception as e:  # noqa: BLE001 -- no reranker: the tools skip the rerank stage
            logger.error(f"Failed to initialize reranker: {e}")
            return None

    def _build_metadata_filters(self, metadata_filters: Optional[dict] = None) -> Optional[dict]:
        """dict -> Chroma where: plain values become $eq, operator dicts pass through, several keys
        are joined by $and (kb_search_toolkit.py:63-96)."""
        if not metadata_filters:
            return None
        parts = [{k: v} if isinstance(v, dict) and any(op.startswith("$") for op in v) else {k: {"$eq": v}}
                 for k, v in metadata_filters.items()]
        if not parts:
            return None
        return parts[0] if len(parts) == 1 else {"$and": parts}

    @staticmethod
    def _row(result, score_key="embedding_score", extra=None):
        d = {"rank": result.rank}
        if extra:
            d.update(extra)
        else:
            d[score_key] = round(result.score, 4)
        d.update({"content": result.chunk.content, "chunk_id": result.chunk.id,
                  "document_id": result.chunk.document_id, "source": result.chunk.metadata.get("source", ""),
                  "metadata": result.chunk.metadata})
        return d

    async def kb_embedding_search(self, kb_id: int, query: str, top_k: Optional[int] = None,
                                  metadata_filters: Optional[dict] = None, auto_rerank: bool = True) -> str:
        if auto_rerank and not self.reranker:
            auto_rerank = False
        try:
            top_k = top_k if top_k is not None else self.default_top_k
            retrieval_top_k = top_k * self.recall_multiplier if auto_rerank else top_k
            filters = self._build_metadata_filters(metadata_filters)
            retriever = await self._create_retriever(kb_id, retrieval_top_k)
            results = await retriever.retrieve(query=query, filters=filters)
            out = {"kb_id": kb_id, "query": query, "total_results": len(results), "top_k": top_k,
                   "filters_applied": metadata_filters if metadata_filters else None,
                   "results": [self._row(r) for r in results]}
            if auto_rerank and results:
                try:
                    emb_scores = {r.chunk.id: r.score for r in results}
                    reranked = await self.reranker.rerank(query=query, results=results, top_k=top_k)
                    out["reranked"] = True
                    out["total_results"] = len(reranked)
                    out["results"] = [self._row(r, extra={"rerank_score": round(r.score, 4), "embedding_score": round(
                        emb_scores.get(r.chunk.id, 0.0), 4)}) for r in reranked]
                except Exception as e:  # noqa: BLE001 -- keep the embedding results
                    logger.warning(f"Auto-rerank failed: {e}, returning embedding results")
                    out["reranked"] = False
                    out["rerank_error"] = str(e)
            else:
                out["reranked"] = False
            return json.dumps(out, ensure_ascii=False, indent=2)
        except Exception as e:  # noqa: BLE001 -- the tools answer errors as JSON (:290-300)
            logger.error(f"KB search failed: {e}")
            return json.dumps({"error": str(e), "kb_id": kb_id, "query": query}, ensure_ascii=False)

    async def kb_rerank(self, query: str, candidates: str, top_k: Optional[int] = None, model: Optional[str] = None,
                        boost_metadata: Optional[dict] = None) -> str:
        try:
            top_k = top_k if top_k is not None else self.default_top_k
            model = model or self.reranker_config.get("model", "jina-reranker-v2-base-multilingual")
            try:
                data = json.loads(candidates)
            except json.JSONDecodeError as e:
                return json.dumps({"error": f"Invalid JSON format in candidates: {str(e)}"}, ensure_ascii=False)
            if "results" not in data:
                return json.dumps({"error": "Missing 'results' field in candidates JSON"}, ensure_ascii=False)
            items = data["results"]
            if len(items) <= 1:
                return candidates
            emb_scores, results = {}, []
            for it in items:
                score = it.get("embedding_score", it.get("score", 0.0))
                emb_scores[it["chunk_id"]] = score
                results.append(RetrievalResult(chunk=Chunk(id=it["chunk_id"], document_id=it["document_id"],
                                                           content=it["content"], chunk_index=0,
                                                           metadata=it.get("metadata", {})),
                                               score=score, rank=it["rank"]))
            reranked = await self.reranker.rerank(query=query, results=results, top_n=top_k)  # (sic, :391-393)
            out = {"kb_id": data.get("kb_id"), "query": query, "total_results": len(reranked),
                   "original_count": len(items), "rerank_top_k": top_k, "rerank_model": model, "reranked": True,
                   "results": [self._row(r, extra={"rerank_score": round(r.score, 4), "embedding_score": round(
                       emb_scores.get(r.chunk.id, 0.0), 4)}) for r in reranked]}
            return json.dumps(out, ensure_ascii=False, indent=2)
        except Exception as e:  # noqa: BLE001
            logger.error(f"Reranking failed: {e}")
            return json.dumps({"error": str(e), "query": query}, ensure_ascii=False)

    async def kb_file_search(self, kb_id: int, query: str, top_k: Optional[int] = None,
                             metadata_filters: Optional[dict] = None, auto_rerank: bool = True,
                             include_summary: bool = True) -> str:
        try:
            top_k = top_k if top_k is not None else self.file_search_top_k
            retrieval_top_k = top_k * self.recall_multiplier if auto_rerank else top_k
            base = self._build_metadata_filters(metadata_filters)
            summary_only = {"index_type": {"$eq": "index_summary"}}
            filters = {"$and": [base, summary_only]} if base else summary_only
            retriever = await self._create_retriever(kb_id, retrieval_top_k)
            results = await retriever.retrieve(query=query, filters=filters)
            files: dict[str, dict] = {}
            hidden = {"index_type", "chunk_index", "_derived_files_etags"}
            for r in results:  # one entry per file: its best summary vector
                name = r.chunk.metadata.get("source", r.chunk.document_id)
                if name in files:
                    continue
                e = {"file_name": name, "relevance_score": r.score, "chunk_id": r.chunk.id, "content": r.chunk.content}
                if include_summary:
                    e["summary"] = r.chunk.metadata.get("summary", "")
                e["metadata"] = {k: v for k, v in r.chunk.metadata.items() if k not in hidden}
                files[name] = e
            ranked = sorted(files.values(), key=lambda x: x["relevance_score"], reverse=True)
            out = {"kb_id": kb_id, "query": query, "total_files": len(ranked), "search_type": "file_level",
                   "index_type": "index_summary", "top_k": top_k,
                   "filters_applied": metadata_filters if metadata_filters else None, "reranked": False, "files": []}

            def plain(entries):
                rows = []
                for i, e in enumerate(entries, 1):
                    row = {"rank": i, "file_name": e["file_name"], "embedding_score": round(e["relevance_score"], 4),
                           "metadata": e["metadata"]}
                    if include_summary:
                        row["summary"] = e.get("summary", "")
                    rows.append(row)
                return rows

            if auto_rerank and len(ranked) > 1:
                try:
                    emb_scores, cands = {}, []
                    for e in ranked:
                        emb_scores[e["chunk_id"]] = e["relevance_score"]
                        cands.append(RetrievalResult(chunk=Chunk(id=e["chunk_id"], document_id=e["file_name"],
                                                                 content=e["content"], chunk_index=-1,
                                                                 metadata=e["metadata"]),
                                                     score=e["relevance_score"], rank=0))
                    reranker = _reranker_from(self.reranker_config.get("backend", "jina"))
                    reranked = await reranker.rerank(query=query, results=cands, top_k=top_k)
                    out["reranked"] = True
                    out["total_files"] = len(reranked)
                    for i, r in enumerate(reranked, 1):
                        row = {"rank": i, "file_name": r.chunk.document_id, "rerank_score": round(r.score, 4),
                               "embedding_score": round(emb_scores.get(r.chunk.id, 0.0), 4),
                               "metadata": r.chunk.metadata}
                        if include_summary:
                            row["summary"] = r.chunk.metadata.get("summary", "")
                        out["files"].append(row)
                except Exception as e:  # noqa: BLE001 -- fall back to the embedding order
                    logger.warning(f"Auto-rerank failed: {e}, returning embedding results")
                    out["reranked"] = False
                    out["rerank_error"] = str(e)
                    out["files"] = plain(ranked[:top_k])
            else:
                out["files"] = plain(ranked[:top_k])
            return json.dumps(out, ensure_ascii=False, indent=2)
        except Exception as e:  # noqa: BLE001
            logger.error(f"File search failed: {e}")
            return json.dumps({"error": str(e), "kb_id": kb_id, "query": query}, ensure_ascii=False)

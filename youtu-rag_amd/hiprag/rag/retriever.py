"""Retrievers over any BaseVectorStore / BaseEmbedder pair.

VectorRetriever keeps the reference's semantics exactly
(utu/rag/knowledge_retrieval/base_retriever.py:14-99):
  * ``top_k`` falls back to config.top_k (:53); ``filters`` / ``similarity_threshold``
    come from kwargs (:54-55);
  * the store is asked for ``2*top_k`` when a reranker is set, else ``top_k`` (:61-63),
    with the keyword call ``query_embedding=``;
  * ranks are the 1-based positions BEFORE threshold filtering (:72), and a
    threshold <= 0 disables filtering (:71);
  * optional rerank, then ``[:top_k]`` (:75-80).
BatchedVectorRetriever overrides batch_retrieve (the reference's loop at :95-98)
with one query-embedding batch and one GPU search launch for the whole batch,
producing the same per-query results.
"""
from __future__ import annotations

import logging

from .base import BaseEmbedder, BaseReranker, BaseRetriever, BaseVectorStore, RetrievalResult
from .config import RetrieverConfig

logger = logging.getLogger(__name__)


class VectorRetriever(BaseRetriever):
    def __init__(self, vector_store: BaseVectorStore, embedder: BaseEmbedder, config: RetrieverConfig | None = None,
                 reranker: BaseReranker | None = None):
        self.vector_store = vector_store
        self.embedder = embedder
        self.config = config or RetrieverConfig()
        self.reranker = reranker
        if self.config.enable_reranking and self.reranker is None:
            # the reference builds RerankerFactory.create(backend="auto", model=config.reranker_model)
            # (base_retriever.py:36-40), an HTTP client; the MI355X replacement is the in-process
            # cross-encoder (local checkpoint if reranker_model is a path, else the seeded preset)
            from .rerankers import RerankerFactory

            self.reranker = RerankerFactory.create(backend="rocm", model_name_or_path=self.config.reranker_model)

    def _to_results(self, hits, threshold: float) -> list[RetrievalResult]:
        out = []
        for pos, (chunk, score) in enumerate(hits):
            if threshold <= 0.0 or score >= threshold:
                out.append(RetrievalResult(chunk=chunk, score=score, rank=pos + 1))
        return out

    async def _finish(self, query: str, results: list[RetrievalResult], top_k: int) -> list[RetrievalResult]:
        if self.reranker and results:
            results = await self.reranker.rerank(query=query, results=results, top_k=top_k)
        return results[:top_k]

    async def retrieve(self, query: str, top_k: int | None = None, **kwargs) -> list[RetrievalResult]:
        top_k = top_k or self.config.top_k
        threshold = kwargs.get("similarity_threshold", self.config.similarity_threshold)
        qv = await self.embedder.embed_query(query)
        hits = await self.vector_store.search(query_embedding=qv, top_k=top_k * 2 if self.reranker else top_k,
                                              filters=kwargs.get("filters"))
        return await self._finish(query, self._to_results(hits, threshold), top_k)

    async def batch_retrieve(self, queries: list[str], top_k: int | None = None, **kwargs
                             ) -> list[list[RetrievalResult]]:
        return [await self.retrieve(query=q, top_k=top_k, **kwargs) for q in queries]


class BatchedVectorRetriever(VectorRetriever):
    """Same results as VectorRetriever, but batch_retrieve embeds all queries at once
    (``embed_queries`` when the embedder has it) and runs one batched search."""

    async def batch_retrieve(self, queries: list[str], top_k: int | None = None, **kwargs
                             ) -> list[list[RetrievalResult]]:
        if not queries:
            return []
        search_batch = getattr(self.vector_store, "search_batch", None)
        if search_batch is None:
            return await super().batch_retrieve(queries, top_k=top_k, **kwargs)
        top_k = top_k or self.config.top_k
        threshold = kwargs.get("similarity_threshold", self.config.similarity_threshold)
        embed_many = getattr(self.embedder, "embed_queries", None)
        qvs = await embed_many(queries) if embed_many else [await self.embedder.embed_query(q) for q in queries]
        hits = search_batch(qvs, top_k * 2 if self.reranker else top_k, kwargs.get("filters"))
        results = [self._to_results(h, threshold) for h in hits]
        rerank_batch = getattr(self.reranker, "rerank_batch", None)
        if rerank_batch is not None:  # one set of cross-encoder batches for every query's pairs
            idx = [i for i, r in enumerate(results) if r]
            try:
                for i, r in zip(idx, rerank_batch([queries[i] for i in idx], [results[i] for i in idx], top_k)):
                    results[i] = r
                return [r[:top_k] for r in results]
            except Exception as e:  # per-query path keeps the reference's failure semantics
                logger.error(f"batched reranking failed ({e}); reranking query by query")
        return [await self._finish(q, r, top_k) for q, r in zip(queries, results)]


class HybridRetriever(BaseRetriever):
    """Delegates to VectorRetriever, as the reference does (base_retriever.py:102-154)."""

    def __init__(self, vector_store: BaseVectorStore, embedder: BaseEmbedder, config: RetrieverConfig | None = None):
        self.vector_retriever = BatchedVectorRetriever(vector_store=vector_store, embedder=embedder, config=config)
        self.config = config or RetrieverConfig()

    async def retrieve(self, query: str, top_k: int | None = None, **kwargs) -> list[RetrievalResult]:
        return await self.vector_retriever.retrieve(query=query, top_k=top_k, **kwargs)

    async def batch_retrieve(self, queries: list[str], top_k: int | None = None, **kwargs
                             ) -> list[list[RetrievalResult]]:
        return await self.vector_retriever.batch_retrieve(queries=queries, top_k=top_k, **kwargs)

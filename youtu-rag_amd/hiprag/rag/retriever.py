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

import asyncio
import logging
import os
import threading
import weakref
from concurrent.futures import ThreadPoolExecutor

from .base import BaseEmbedder, BaseReranker, BaseRetriever, BaseVectorStore, RetrievalResult
from .config import RetrieverConfig

logger = logging.getLogger(__name__)


class _Cohort:
    """One event loop's waiting retrieve calls and whether its drain is running."""

    __slots__ = ("pending", "running", "__weakref__")

    def __init__(self):
        self.pending: list = []
        self.running = False


class _FusedRetrieve:
    """Concurrent ``retrieve`` calls (base_retriever.py:53-63: embed_query, then store.search) as cohorts of up to
    ``max_batch`` queries, each cohort ONE embedder forward whose (B, dim) output stays on the GPU and goes straight
    into ONE store search (HipVectorStore.search_device_sync) -- no per-query vector lists through the host, no
    second batching stage, and the cohort's forward and FILTER run back to back on one stream instead of
    interleaving with other cohorts' work.  A worker thread runs the forward + search; the Chunk objects are built
    on the caller's loop.  Results are those of the two-step path for the same vectors (the same store search;
    embed_query returns this forward's rows as lists).  Each event loop has its own queue and drain (futures are
    resolved only on their own loop); the loops share the one worker."""

    def __init__(self, retriever: "VectorRetriever", max_batch: int):
        self.r, self.max_batch = retriever, max(1, int(max_batch))
        self._queues: "weakref.WeakKeyDictionary" = weakref.WeakKeyDictionary()
        self._qlock = threading.Lock()
        self._pool = None
        self._pool_lock = threading.Lock()
        self.cohorts = 0  # diagnostics: cohorts run / queries through them
        self.queries = 0

    def submit(self, query: str, top_k: int, threshold: float) -> asyncio.Future:
        loop = asyncio.get_running_loop()
        fut = loop.create_future()
        with self._qlock:
            c = self._queues.get(loop)
            if c is None:
                c = self._queues[loop] = _Cohort()
        c.pending.append((query, int(top_k), float(threshold), fut))
        if not c.running:
            c.running = True
            loop.call_soon(lambda: loop.create_task(self._drain(c)))
        return fut

    def _executor(self):
        with self._pool_lock:
            if self._pool is None:
                self._pool = ThreadPoolExecutor(max_workers=1, thread_name_prefix="hiprag-retrieve")
            return self._pool

    def _run(self, texts: list[str], k: int):
        """Worker thread: the cohort's forward and its search (device queries), the host records back."""
        # (the embedder's forwards take its lock themselves: graph inputs are shared with its other callers)
        q = self.r.embedder.encode_queries(texts)
        return self.r.vector_store.search_device_sync(q, k)

    async def _drain(self, c: _Cohort):
        loop = asyncio.get_running_loop()
        batch: list = []
        try:
            while c.pending:
                batch, c.pending = c.pending[: self.max_batch], c.pending[self.max_batch:]
                batch = [e for e in batch if not e[3].done()]
                if not batch:
                    continue
                k = max(e[1] for e in batch)
                try:
                    ran = await loop.run_in_executor(self._executor(), self._run, [e[0] for e in batch], k)
                    hits = self.r.vector_store._assemble(([None] * len(batch), k, None), ran)
                except Exception as exc:  # noqa: BLE001 -- this cohort's callers see the failure
                    for e in batch:
                        if not e[3].done():
                            e[3].set_exception(exc)
                    batch = []
                    continue
                self.cohorts += 1
                self.queries += len(batch)
                for (_, kq, th, f), h in zip(batch, hits):
                    if not f.done():
                        f.set_result(self.r._to_results(h[:kq], th))
                batch = []
        except BaseException as exc:  # the drain itself stopped (loop shutdown): no caller is left waiting
            err = exc if isinstance(exc, Exception) else RuntimeError(f"retrieval stopped: {exc!r}")
            for e in batch + c.pending:
                if not e[3].done():
                    e[3].set_exception(err)
            c.pending = []
            raise
        finally:
            c.running = False

    def close(self):
        with self._pool_lock:
            if self._pool is not None:
                self._pool.shutdown(wait=True)
                self._pool = None


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
        # the fused path (one forward + one device-query search per cohort of concurrent calls) where both halves are
        # hiprag's: the in-process embedder and the HIP store; anything else keeps the reference's two awaits
        self._fused = _FusedRetrieve(self, getattr(embedder, "batch_size", 64)) if self._fusable() else None

    def _fusable(self) -> bool:
        if os.environ.get("HIPRAG_FUSED_RETRIEVE", "1") == "0":  # (A/B switch: the reference's two awaits)
            return False
        return (self.reranker is None and callable(getattr(self.vector_store, "search_device_sync", None))
                and callable(getattr(self.embedder, "encode_queries", None))
                and hasattr(self.embedder, "_fwd_lock") and getattr(self.embedder, "fused_retrieve", True))

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
        if self._fused is not None and not kwargs.get("filters") and self.reranker is None:
            return await self._fused.submit(query, top_k, threshold)
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

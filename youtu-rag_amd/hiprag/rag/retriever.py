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
import time
import weakref

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
    into ONE store search -- no per-query vector lists through the host, no second batching stage.

    One worker thread pipelines the cohorts: it enqueues cohort i+1's forward and its search (the pipelined shard
    search of hiprag.dist.ShardedSearch on the store's index: scan + tail streams, guard flags copied asynchronously)
    BEFORE it waits for cohort i's results, so the GPU always has the next cohort queued behind the current one while
    the host tokenises, finalizes and hands results back.  The store's lock is held from a cohort's submit to its
    finalize (a mutation must not move rows under a search in flight).  The Chunk objects are built on the caller's
    loop.  Results are those of the two-step path for the same vectors (the same exact search).  Each event loop has
    its own queue and drain (futures are resolved on their own loop only)."""

    def __init__(self, retriever: "VectorRetriever", max_batch: int):
        import queue

        self.r, self.max_batch = retriever, max(1, int(max_batch))
        self._queues: "weakref.WeakKeyDictionary" = weakref.WeakKeyDictionary()
        self._qlock = threading.Lock()
        self._work: "queue.Queue" = queue.Queue()  # cohorts from every loop, to the worker
        self._thread = None
        self._tlock = threading.Lock()
        self._searcher = None  # (index, ShardedSearch) of the store's current index
        self._k = 0  # the current cohort's largest top_k (worker thread)
        self.cohorts = 0  # diagnostics: cohorts run / queries through them / cohorts overlapped with the next
        self.queries = 0
        self.pipelined = 0
        # diagnostics (worker thread, seconds): forward tokenise + launch, search submit, finalize (the device wait
        # included), and cohorts finalized with no next cohort queued behind them (pipeline bubbles)
        self.timing = {"encode": 0.0, "submit": 0.0, "finalize": 0.0, "bubbles": 0}

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
            loop.call_soon(self._form, c, loop)
        return fut

    def _form(self, c: _Cohort, loop):
        """On the loop, one iteration after the first call: hand the waiting calls to the worker in cohorts."""
        c.running = False
        while c.pending:
            batch, c.pending = c.pending[: self.max_batch], c.pending[self.max_batch:]
            batch = [e for e in batch if not e[3].done()]
            if batch:
                self._work.put((loop, batch))  # (before the check: a worker that is just leaving sees it)
                self._ensure_worker()

    def _ensure_worker(self):
        with self._tlock:
            if self._thread is None or not self._thread.is_alive():
                self._thread = threading.Thread(target=self._worker, name="hiprag-retrieve", daemon=True)
                self._thread.start()

    # ---- worker thread
    def _search(self, q):
        """Launch the cohort's search (store lock held by the caller).  Returns a finisher -> (raw, tables)."""
        store = self.r.vector_store
        tables = (store._records, store._metas, store._epoch)
        idx, n_live = store._index, store.count_sync()
        B, k = q.shape[0], self._k
        if idx is None or n_live == 0 or k <= 0:
            return lambda: (None, tables)
        k = min(k, n_live)
        ss = self._sharded(idx, B) if q.is_cuda else None
        if ss is None:  # (CPU tests, multi-device handles, k beyond the pipelined path: the synchronous search)
            ran = store.search_device_sync(q, k)
            return lambda: ran
        slot = ss.submit(q, k)

        def finish():
            s_out, r_out = ss.finalize(slot)
            return (s_out.cpu().numpy(), r_out.cpu().numpy()), tables
        return finish

    def _sharded(self, idx, B):
        from .. import _native

        if not hasattr(idx, "search_shard") or len(getattr(idx, "devices", (0,))) > 1 or self._k > _native.HR_MAX_K:
            return None
        if self._searcher is None or self._searcher[0] is not idx or self._searcher[1].max_batch < B:
            import torch

            from ..dist import ShardedSearch

            self._drop_searcher()
            dev = torch.device("cuda", idx.device)
            self._searcher = (idx, ShardedSearch(idx, 0, max_batch=max(B, self.max_batch), device=dev, max_k=16))
        return self._searcher[1]

    def _deliver(self, loop, batch, ran, exc=None):
        """Back on the caller's loop: Chunks from the finished search, each call's top_k and threshold."""
        if exc is None:
            try:
                res = self.r.vector_store._assemble_results(ran, [e[1] for e in batch], [e[2] for e in batch],
                                                            RetrievalResult)
            except Exception as e:  # noqa: BLE001
                exc = e
        for i, (_, kq, th, f) in enumerate(batch):
            if f.done():
                continue
            if exc is not None:
                f.set_exception(exc)
            else:
                f.set_result(res[i])

    def _post(self, loop, batch, ran, exc=None):
        if loop.is_closed():
            return  # (the caller's loop ended: nobody waits for these)
        try:
            loop.call_soon_threadsafe(self._deliver, loop, batch, ran, exc)
        except RuntimeError:  # closed between the check and the call
            pass

    def _worker(self):
        import queue

        store = self.r.vector_store
        inflight = None  # (loop, batch, finisher) of the cohort whose search is on the GPU
        locked = False
        while True:
            try:
                item = self._work.get(timeout=0.5) if inflight is None else self._work.get_nowait()
            except queue.Empty:
                item = None
            if item is None and inflight is None:
                with self._tlock:  # (under the lock _ensure_worker takes: a cohort put now starts a new worker)
                    if self._work.empty():
                        self._thread = None
                        return  # idle: the thread ends
                continue
            nxt = None
            tm = self.timing
            if item is not None:
                loop, batch = item
                try:
                    self._k = max(e[1] for e in batch)
                    t0 = time.perf_counter()
                    q = self.r.embedder.encode_queries([e[0] for e in batch])  # (device, enqueued)
                    t1 = time.perf_counter()
                    if not locked:
                        store._lock.acquire()
                        locked = True
                    nxt = (loop, batch, self._search(q))
                    tm["encode"] += t1 - t0
                    tm["submit"] += time.perf_counter() - t1
                except Exception as e:  # noqa: BLE001 -- this cohort's callers see the failure
                    self._post(loop, batch, None, e)
            if inflight is not None:
                loop0, batch0, finish = inflight
                if nxt is None:
                    tm["bubbles"] += 1
                t0 = time.perf_counter()
                try:
                    ran = finish()
                    self._post(loop0, batch0, ran)
                except Exception as e:  # noqa: BLE001
                    self._post(loop0, batch0, None, e)
                tm["finalize"] += time.perf_counter() - t0
                self.cohorts += 1
                self.queries += len(batch0)
                if nxt is not None:
                    self.pipelined += 1
            inflight = nxt
            if inflight is None and locked:
                store._lock.release()
                locked = False

    def _drop_searcher(self):
        """Release the pipelined searcher of a previous index (nothing is in flight: the worker finalizes every
        cohort before it takes the next index); a store that closed its index already released what it held."""
        if self._searcher is None:
            return
        idx, ss = self._searcher
        self._searcher = None
        if getattr(idx, "_h", None):
            ss.close()

    def close(self):
        t = self._thread
        if t is not None:
            t.join(timeout=10)
        self._drop_searcher()


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
                and callable(getattr(self.vector_store, "_assemble_results", None))
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

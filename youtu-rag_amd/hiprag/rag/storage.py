"""HipVectorStore: the reference's BaseVectorStore served by the MI355X index.

Drop-in for ChromaVectorStore (utu/rag/storage/implementations/chroma_store.py,
the production store) with the exact-search semantics of FAISSVectorStore
(faiss_store.py):
  * add_chunks (chroma :64-88): metadata stored as {document_id, chunk_index,
    **non-None chunk.metadata}; ids already present are skipped with a warning,
    ids repeated inside one call raise ValueError (Chroma DuplicateIDError);
  * search (chroma :90-148): exact top-k on the GPU; cosine/"dot" similarity =
    inner product (faiss :179-180; chroma's 1 - distance :135 for those spaces),
    "euclidean" similarity = 1 - squared L2 distance (chroma's "l2" space, :48-53);
    ``filters`` are compiled to a row bitmap (plain dict or Chroma where-clause,
    filters.py: cached per predicate) and applied inside the scan, i.e. exact top-k
    among matching rows;
  * delete / delete_by_document_id / delete_by_metadata (chroma :150-222):
    row tombstones in the index + removal from the host tables;
  * get_by_id (chroma :224-247); count / clear / delete_collection.

Concurrency (SURVEY §7 hard part 5).  The reference calls Chroma synchronously inside
``async def`` (chroma_store.py:118) and its callers issue one query per
``VectorRetriever.retrieve`` (base_retriever.py:58-63).  Here ``search`` hands the query
to a micro-batcher: every ``search`` awaiting at the same time (same filter) becomes ONE
GPU launch, run in a worker thread (``asyncio.to_thread``; ctypes drops the GIL), so the
event loop keeps running and concurrent retrievers share one corpus pass.  Requests that
arrive while a launch is in flight form the next batch (no timer: the batch size follows
the load).  Results are identical to sequential calls (top-k of a smaller k is the prefix of
the larger k's, order score desc / row asc).

Embeddings: the index keeps the normalised vectors in ``dtype``: fp32 by default, what the
reference stores (faiss_store.py:98; Chroma float32), so rankings and scores are the reference's.
``dtype: bf16`` (opt-in) halves the bytes per row and doubles the scan rate; search is then exact
over the stored bf16 values, whose ranking departs from the fp32 answer where two rows' scores lie
within the bf16 rounding of their dot products: recall@10 against the exact fp32 top-10 measured
0.99 at 1M-10M rows (bench.py ``recall_at_10_vs_fp32``, tests/test_gpu_scale.py).  Chroma returns the raw fp32
embedding it stored (chroma_store.py:233-244): ``keep_embeddings: true`` keeps a host fp32
copy for ``get_by_id`` / ``include_embeddings``; without it they return the stored
(normalised, quantised) row.

Persistence: generation snapshots + an append-only journal (persist.py); ``add_chunks`` and
``delete*`` write O(chunk) bytes.  ``index_params.devices`` (list of GPU ids) shards the rows
of one collection over several GPUs inside one handle (hr_index_create with n_dev > 1).
"""
from __future__ import annotations

import asyncio
import contextlib
import json
import logging
import os
import threading
from array import array
from collections import deque
from typing import Any

import numpy as np

from .. import _native
from . import filters as F
from . import persist as P
from .base import BaseVectorStore, Chunk
from .config import VectorStoreConfig

try:  # the per-hit result assembly in C (csrc/host/hostfast.c, built by csrc/Makefile); host-side only, same output
    from . import _hostfast
except ImportError:  # pragma: no cover - a source tree without the build: the Python loop below
    _hostfast = None


def _assemble_py(C, rec_l, meta_l, score_l, per_q, embs, untrack=False):
    """The per-query (Chunk, score) lists of a batch's gathered hits; _hostfast.assemble is the same in C
    (`untrack` only applies there)."""
    out, i = [], 0
    for cnt in per_q:  # one pass: each query's hits straight into its list
        res = []
        for j in range(i, i + cnt):
            r = rec_l[j]
            if r is None:
                continue
            m = meta_l[j]
            res.append((C(r[0], m.get("document_id", ""), r[2], m.get("chunk_index", 0), dict(m),
                          None if embs is None else embs[j]), score_l[j]))
        out.append(res)
        i += cnt
    return out


def _assemble_results_py(C, R, rec_l, meta_l, score_l, per_q, embs, ks, ths, untrack=False):
    """The per-query RetrievalResult lists of a batch's gathered hits for calls with top_k ks[q] and similarity
    threshold ths[q] (VectorRetriever._to_results over _assemble_py's pairs cut to top_k); _hostfast.assemble_results
    is the same in C (`untrack` only applies there)."""
    out, i = [], 0
    for q, cnt in enumerate(per_q):
        res, pos, kq, th = [], 0, ks[q], ths[q]
        for j in range(i, i + cnt):
            r = rec_l[j]
            if r is None or pos >= kq:
                continue
            pos += 1
            if th > 0.0 and not score_l[j] >= th:
                continue
            m = meta_l[j]
            res.append(R(C(r[0], m.get("document_id", ""), r[2], m.get("chunk_index", 0), dict(m),
                           None if embs is None else embs[j]), score_l[j], pos))
        out.append(res)
        i += cnt
    return out


logger = logging.getLogger(__name__)

_METRIC = {"cosine": "cosine", "dot": "ip", "euclidean": "l2"}


class _ObjColumn:
    """A growable per-row column of Python objects in a numpy object array.  Used instead of a list for
    the 10M-entry host tables: an object ndarray is not tracked by Python's cycle collector, a list is,
    and every full collection walked the lists' 10M entries (~0.1 s each; p99 search latency under
    load 600 ms without it, 6-70 ms with it -- tools/bench_async.py).  Holds only acyclic values."""

    __slots__ = ("a", "n")

    def __init__(self, values=()):
        values = list(values)
        self.a = np.empty(max(1024, len(values)), object)
        for i, v in enumerate(values):  # element-wise: tuples must stay objects, not become array rows
            self.a[i] = v
        self.n = len(values)

    def __len__(self):
        return self.n

    def __getitem__(self, i):
        return self.a[i]

    def __setitem__(self, i, v):
        self.a[i] = v

    def __iter__(self):
        return iter(self.a[: self.n])

    def append(self, v):
        if self.n == len(self.a):
            grown = np.empty(2 * len(self.a), object)
            grown[: self.n] = self.a
            self.a = grown
        self.a[self.n] = v
        self.n += 1


class _SearchBatcher:
    """Coalesces concurrent ``search`` calls into batched launches (one per filter group).

    Up to ``depth`` launches are in flight, and the Chunk objects of a finished batch are assembled on the
    event-loop thread while the next launch runs.  An unfiltered batch on a single-device index is launched
    from the event loop itself through the library's asynchronous entry point
    (hr_index_search_submit_host: the call only enqueues the GPU work and returns); its completion arrives
    as a count on an eventfd the loop watches (written by a host function behind the batch's results), so
    no Python thread takes part -- no GIL hand-off between a worker and the loop per launch.  Filtered
    batches, multi-device handles, and launches that find the handle or the store busy run the blocking
    search in a worker thread (``asyncio.to_thread``; ctypes drops the GIL)."""

    def __init__(self, store: "HipVectorStore", max_batch: int, depth: int = 2):
        self.store, self.max_batch, self.depth = store, max(1, int(max_batch)), max(1, int(depth))
        self.pending: list = []
        self.running = False
        self.launches = 0         # diagnostics
        self.native_launches = 0  # ... of which through the asynchronous native entry point
        self.efd = -1             # eventfd of native completions (one count per finished batch)
        self._native: deque = deque()  # completion futures of native launches, in submission order
        self._loop = None         # the loop the eventfd reader is registered with
        self._drain_loop = None   # the loop the running drain belongs to
        self._inflight: dict = {}  # the running drain's launches: awaitable -> (batch, prep, native info or None)

    def submit(self, q: np.ndarray, top_k: int, filters) -> asyncio.Future:
        """Queue one query; the future resolves to its (Chunk, score) list.  A plain call, not a coroutine: the
        caller's own coroutine awaits the future, so a query in flight holds one coroutine frame fewer for the
        cycle collector to walk and promote (the store's event loop is collector-bound under load)."""
        dim = self.store.dim
        if dim is not None and q.shape[0] != dim:  # checked before queueing: a bad query fails alone
            raise ValueError(f"query dim {q.shape[0]} != collection dim {dim}")
        loop = asyncio.get_running_loop()
        if self._drain_loop is not None and self._drain_loop is not loop and self._drain_loop.is_closed():
            self._recover_from_closed_loop(loop)
        fut = loop.create_future()
        self.pending.append((q, int(top_k), filters, _filter_key(filters), fut))
        if not self.running:
            self.running, self._drain_loop = True, loop
            # start draining on the next loop iteration: every task that is ready now enqueues first
            loop.call_soon(lambda: loop.create_task(self._drain()))
        return fut

    def _recover_from_closed_loop(self, loop):
        """The loop that ran the last drain has closed -- possibly under it (asyncio.run ending with searches queued
        or in flight: the drain never ran, or was cancelled with native launches outstanding): finish those
        native launches here (blocking collects: their slots free, results dropped -- nobody waits for them), drop
        their completion counts from the eventfd, forget the dead loop's queries and start afresh on `loop`."""
        for _batch, _prep, info in list(self._inflight.values()):
            if info is not None:
                with contextlib.suppress(Exception):
                    self.store._collect_native(info, blocking=True)
        self._inflight = {}
        if self.efd >= 0:
            with contextlib.suppress(BlockingIOError, OSError):
                os.eventfd_read(self.efd)  # (the collects waited for every notify of those launches)
        self._native.clear()
        self._loop = None  # its reader went with the closed loop; native_fd registers one with `loop`
        self.pending = [e for e in self.pending if e[4].get_loop() is loop]
        self.running, self._drain_loop = False, None

    def _take(self):
        key = self.pending[0][3]
        batch, rest = [], []
        for e in self.pending:
            (batch if e[3] == key and len(batch) < self.max_batch else rest).append(e)
        self.pending = rest
        return batch

    @staticmethod
    def _fail(batch, exc):
        for e in batch:
            if not e[4].done():
                e[4].set_exception(exc)

    # -- native completions
    def native_fd(self, loop) -> int:
        """The eventfd native launches signal, its reader registered with `loop` (-1: unavailable)."""
        if self.efd < 0:
            if not hasattr(os, "eventfd"):
                return -1
            self.efd = os.eventfd(0, os.EFD_NONBLOCK | os.EFD_CLOEXEC)
        if self._loop is not loop:
            loop.add_reader(self.efd, self._on_completions)
            self._loop = loop
        return self.efd

    def _on_completions(self):
        try:
            n = os.eventfd_read(self.efd)
        except BlockingIOError:
            return
        for _ in range(n):  # batches finish in submission order (one stream)
            if not self._native:
                break
            fut = self._native.popleft()
            if not fut.done():
                fut.set_result(None)

    def _release_loop(self):
        if self._loop is not None and not self._native:
            with contextlib.suppress(Exception):
                self._loop.remove_reader(self.efd)
            self._loop = None

    def close(self):
        self._release_loop()
        if self.efd >= 0 and not self._native:
            os.close(self.efd)
            self.efd = -1

    def _launch(self, loop, prep):
        """Start one batch: (awaitable, info).  info is None for a worker-thread launch (the awaitable's
        result is the search), else the native launch to collect once the awaitable resolves."""
        info = self.store._submit_native(prep, self, loop)
        if info is not None:
            fut = loop.create_future()
            self._native.append(fut)
            self.native_launches += 1
            return fut, info
        return asyncio.ensure_future(asyncio.to_thread(self.store._run_search, prep)), None

    async def _drain(self):
        loop = asyncio.get_running_loop()
        inflight: dict = {}  # awaitable -> (batch, prep, native launch info or None)
        self._inflight = inflight  # (seen by _recover_from_closed_loop if this loop closes under the drain)
        batch: list = []
        try:
            while self.pending or inflight:
                while self.pending and len(inflight) < self.depth:
                    batch = self._take()
                    try:
                        qs = np.stack([e[0] for e in batch])
                        k = max(e[1] for e in batch)
                        self.launches += 1
                        prep = self.store._prep_search(qs, k, batch[0][2])
                        aw, info = self._launch(loop, prep)
                    except Exception as exc:  # noqa: BLE001 -- this batch's waiters see the failure
                        self._fail(batch, exc)
                        continue
                    inflight[aw] = (batch, prep, info)
                batch = []
                if not inflight:
                    continue
                done, _ = await asyncio.wait(list(inflight), return_when=asyncio.FIRST_COMPLETED)
                for aw in done:
                    batch, prep, info = inflight.pop(aw)
                    try:
                        if info is None:
                            ran = aw.result()
                        else:
                            ran = self.store._collect_native(info, blocking=False)
                            if ran is None:  # the store is busy (a mutation holds its lock): collect in a worker
                                t = asyncio.ensure_future(asyncio.to_thread(self.store._collect_native, info, True))
                                inflight[t] = (batch, prep, None)
                                batch = []
                                continue
                        res = self.store._assemble(prep, ran)
                    except Exception as exc:  # noqa: BLE001 -- every waiter sees the failure
                        self._fail(batch, exc)
                        continue
                    for e, r in zip(batch, res):
                        if not e[4].done():
                            e[4].set_result(r if len(r) <= e[1] else r[: e[1]])
                batch = []
        except BaseException as exc:  # never leave a waiter hanging: fail what this drain holds
            err = exc if isinstance(exc, Exception) else RuntimeError(f"search batcher stopped: {exc!r}")
            self._fail(batch, err)
            for b, _, _ in inflight.values():
                self._fail(b, err)
            raise
        finally:
            self.running = False
            self._release_loop()


def _filter_key(filters) -> str:
    if not filters:
        return ""
    return json.dumps(filters, sort_keys=True, default=repr)


class HipVectorStore(BaseVectorStore):
    def __init__(self, config: VectorStoreConfig, *, index_factory=None, index_loader=None):
        self.config = config
        params = dict(config.index_params or {})
        self.dtype = params.get("dtype", "f32")  # the reference's store dtype; bf16 is an opt-in
        devs = params.get("devices")
        self.devices = [int(d) for d in devs] if devs else [int(params.get("device", 0))]
        self.device = self.devices[0]
        self.capacity = int(params.get("capacity", 0))
        self.include_embeddings = bool(params.get("include_embeddings", False))
        self.keep_embeddings = bool(params.get("keep_embeddings", False))
        # returned Chunks with atomic-valued metadata left off the cycle collector (faster under heavy load; a cycle
        # a caller later builds through such a Chunk is then never collected).  Off: ordinary tracked objects.
        self.untracked_results = bool(params.get("untracked_results", False))
        self.persist = bool(params.get("persist", True))
        self.fsync = bool(params.get("fsync", True))
        self.journal_fraction = float(params.get("journal_fraction", 0.25))
        self.metric = _METRIC[config.distance_metric]
        if self.dtype not in _native.DTYPES:
            raise ValueError(f"unknown index dtype {self.dtype!r}")
        self._factory = index_factory or (lambda dim: _native.NativeIndex(dim, self.dtype, self.metric,
                                                                          devices=self.devices))
        self._loader = index_loader or (lambda path, dim, dtype, metric: _native.NativeIndex.load(
            path, devices=self.devices, dim=dim, dtype=dtype, metric=metric))
        self._batcher = _SearchBatcher(self, int(params.get("max_batch", 64)), int(params.get("search_depth", 2)))
        # unfiltered batches launched from the event loop through the asynchronous native entry point
        self.native_async = bool(params.get("native_async", True))
        self._lock = threading.RLock()
        self._paths = P.Paths(config.persist_directory, config.collection_name)
        self._gen = 0
        self._journal: P.Journal | None = None
        self._snapshot_bytes = 0
        self._reset_tables()
        if self.persist:
            self._load_if_present()

    def _reset_tables(self):
        # bumped on every reset (clear / delete_collection): a search that ran against the previous
        # tables must not resolve its rows through the new ones
        self._epoch = getattr(self, "_epoch", 0) + 1
        self._index = None
        self.dim: int | None = None
        # host tables, one entry per index row (None = deleted): a tuple of atoms (id, document_id, content,
        # chunk_index) and the stored metadata dict.  Kept apart on purpose: a tuple of atoms and a dict of
        # atoms are untracked by Python's cycle collector, a record dict holding a dict is not -- at 10M
        # rows every full collection then walked 20M+ objects (seconds-long pauses under load)
        self._records = _ObjColumn()  # per row: (id, document_id, content, chunk_index) or None
        self._metas = _ObjColumn()    # per row: the stored metadata dict or None
        self._id_to_row: dict[str, int] = {}
        self._doc_rows: dict[str, array] = {}  # document -> its rows (array('q'): not GC-tracked either)
        self._cols = F.MetadataColumns()
        self._live = np.zeros(0, bool)
        self._raw = None  # keep_embeddings: (capacity, dim) fp32 host copy
        self._defer, self._dirty = 0, False

    # ---------------------------------------------------------------- persistence
    def _load_if_present(self):
        pt = self._paths
        if os.path.exists(pt.manifest):
            with open(pt.manifest) as f:
                man = json.load(f)
            g = int(man["gen"])
            idx_path, rows_path, emb_path = pt.gen(g, "hri"), pt.gen(g, "rows.jsonl"), pt.gen(g, "emb.npy")
            self._gen = g
        else:
            idx_path, rows_path = pt.legacy  # round-1 layout
            emb_path, man = None, None
            if not (os.path.exists(idx_path) and os.path.exists(rows_path)):
                return
        header, records = P.read_rows(rows_path)
        self.dim = int(header["dim"])
        self.dtype, self.metric = header["dtype"], header["metric"]  # the files' own, not the config's
        self._index = self._loader(idx_path, self.dim, self.dtype, self.metric)
        n_idx = self._index.size()[0]
        n_hdr = int(header.get("n_rows", len(records)))
        if not (n_idx == n_hdr == len(records)) or (man is not None and int(man["n_rows"]) != n_idx):
            self._index.close()
            self._index = None
            raise RuntimeError(f"collection files disagree on the row count (index {n_idx}, rows header {n_hdr}, "
                               f"records {len(records)}); refusing to load {rows_path}")
        raw = None
        if self.keep_embeddings and emb_path and os.path.exists(emb_path):
            raw = np.load(emb_path, allow_pickle=False)
        self._install(records, raw)
        self._snapshot_bytes = os.path.getsize(idx_path)
        if man is not None:  # replay the journal of this generation
            n_ops = 0
            for op, a, b in P.Journal.replay(pt.gen(self._gen, "journal")):
                if op == "add":
                    first = self._index.add(b)
                    if first != len(self._records):
                        raise RuntimeError("journal replay: row numbering diverged")
                    self._append_tables(a, b)
                else:
                    self._remove_tables(a.tolist(), journal=False)
                n_ops += 1
            if n_ops:
                logger.info("replayed %d journal entries", n_ops)
        logger.info("loaded %d chunks from %s", len(self._id_to_row), idx_path)

    @staticmethod
    def _split_record(rec: dict | None):
        if rec is None:
            return None, None
        return (rec["id"], rec["document_id"], rec["content"], rec.get("chunk_index", 0)), rec.get("metadata", {})

    def record(self, row: int) -> dict | None:
        """The stored record of a row as the persisted dict (None if deleted)."""
        t = self._records[row]
        if t is None:
            return None
        return {"id": t[0], "document_id": t[1], "content": t[2], "chunk_index": t[3], "metadata": self._metas[row]}

    def _install(self, records: list, raw):
        split = [self._split_record(rec) for rec in records]
        self._records = _ObjColumn(t for t, _ in split)
        self._metas = _ObjColumn(m for _, m in split)
        del split
        self._live = np.array([r is not None for r in records], bool)
        for row, rec in enumerate(self._records):
            if rec is not None:
                self._id_to_row[rec[0]] = row
                self._doc_rows.setdefault(rec[1], array("q")).append(row)
        self._cols.append([m or {} for m in self._metas])
        if self.keep_embeddings:
            self._raw = np.zeros((max(len(records), 1024), self.dim), np.float32)
            if raw is not None and len(raw) == len(records):
                self._raw[: len(records)] = raw

    @contextlib.contextmanager
    def deferred_save(self):
        """Write one snapshot at the end of a block of adds/deletes (bulk ingest) instead of
        journaling each call."""
        self._defer += 1
        try:
            yield self
        finally:
            self._defer -= 1
            if self._defer == 0 and self._dirty:
                self.flush()

    def flush(self):
        """Write a new snapshot generation now (folds the journal in)."""
        with self._lock:
            self._dirty = False
            if not self.persist or self._index is None:
                return
            pt = self._paths
            os.makedirs(self.config.persist_directory, exist_ok=True)
            g = self._gen + 1
            n = len(self._records)
            self._index.save(pt.gen(g, "hri"))
            P.write_rows(pt.gen(g, "rows.jsonl"), {"format": P.FORMAT, "gen": g, "n_rows": n, "dim": self.dim,
                                                  "dtype": self.dtype, "metric": self.metric},
                         (self.record(r) for r in range(n)))
            if self.keep_embeddings:
                P.fsync_write(pt.gen(g, "emb.npy"), writer=lambda f: np.save(f, self._raw[:n], allow_pickle=False))
            P.fsync_write(pt.manifest, json.dumps({"format": P.FORMAT, "gen": g, "n_rows": n, "dim": self.dim,
                                                   "dtype": self.dtype, "metric": self.metric}).encode())
            old = self._gen
            if self._journal is not None:
                self._journal.close()
                self._journal = None
            self._gen = g
            self._snapshot_bytes = os.path.getsize(pt.gen(g, "hri"))
            for f in P.Paths(self.config.persist_directory, self.config.collection_name).all_files():
                if f.startswith(pt.base + f".g{old}.") or f in pt.legacy:
                    with contextlib.suppress(OSError):
                        os.remove(f)

    def _log(self, op: str, rows=None, records=None, vectors=None):
        """Persist one mutation: journal it, or mark the deferred block dirty."""
        if not self.persist or self._index is None:
            return
        if self._defer or self._gen == 0:  # (no snapshot yet: the first write is a snapshot)
            self._dirty = True
            if not self._defer:
                self.flush()
            return
        if self._journal is None:
            self._journal = P.Journal(self._paths.gen(self._gen, "journal"), fsync=self.fsync)
        if op == "add":
            self._journal.append_add(records, vectors)
        else:
            self._journal.append_delete(rows)
        if self._journal.size > max(64 << 20, self.journal_fraction * self._snapshot_bytes):
            self.flush()

    # ---------------------------------------------------------------- writes
    def _fresh(self, chunks: list[Chunk]) -> list[int]:
        """Indices of chunks whose id is not stored yet (chroma skips existing ids, chroma_store.py:64-88)."""
        ids = [c.id for c in chunks]
        if len(set(ids)) != len(ids):
            raise ValueError("duplicate chunk ids inside one add_chunks call")
        keep = [i for i, c in enumerate(chunks) if c.id not in self._id_to_row]
        if len(keep) < len(chunks):
            logger.warning("skipping %d chunk(s) whose id already exists", len(chunks) - len(keep))
        return keep

    def _ensure_index(self, dim: int):
        if self._index is None:
            self.dim = int(dim)
            self._index = self._factory(self.dim)
            if self.capacity:
                self._index.reserve(self.capacity)
        elif dim != self.dim:
            raise ValueError(f"embedding dim {dim} != collection dim {self.dim}")

    @staticmethod
    def _record(c: Chunk) -> dict:
        meta = {"document_id": c.document_id, "chunk_index": c.chunk_index,
                **{k: v for k, v in (c.metadata or {}).items() if v is not None}}
        return {"id": c.id, "document_id": c.document_id, "content": c.content, "chunk_index": c.chunk_index,
                "metadata": meta}

    def _append_tables(self, records: list[dict], vectors: np.ndarray | None):
        first = len(self._records)
        for i, rec in enumerate(records):
            t, m = self._split_record(rec)
            self._records.append(t)
            self._metas.append(m)
            if rec is not None:
                self._id_to_row[rec["id"]] = first + i
                self._doc_rows.setdefault(rec["document_id"], array("q")).append(first + i)
        self._cols.append([(rec or {}).get("metadata", {}) for rec in records])
        n = len(self._records)
        if len(self._live) < n:
            live = np.zeros(max(n, 2 * len(self._live), 1024), bool)
            live[: len(self._live)] = self._live
            self._live = live
        self._live[first:n] = [rec is not None for rec in records]
        if self.keep_embeddings:
            if self._raw is None or len(self._raw) < n:
                raw = np.zeros((max(n, 2 * (0 if self._raw is None else len(self._raw)), 1024), self.dim), np.float32)
                if self._raw is not None:
                    raw[: len(self._raw)] = self._raw
                self._raw = raw
            if vectors is not None:
                self._raw[first:n] = vectors

    def _register(self, fresh: list[Chunk], first: int, vectors: np.ndarray | None):
        records = [self._record(c) for c in fresh]
        if first != len(self._records):
            raise RuntimeError(f"index row {first} != host table size {len(self._records)}")
        self._append_tables(records, vectors)
        self._log("add", records=records, vectors=vectors)
        logger.info("added %d chunks to %s", len(fresh), self.config.collection_name)

    # The async mutators and get_by_id take the store lock in a worker thread: a search launch holds it
    # for a whole GPU pass, and the event loop (where the batcher assembles results) must never wait on it.
    async def add_chunks(self, chunks: list[Chunk]) -> None:
        if not chunks:
            return
        await asyncio.to_thread(self.add_chunks_sync, chunks)

    def add_chunks_sync(self, chunks: list[Chunk]) -> None:
        if not chunks:
            return
        with self._lock:
            fresh = [chunks[i] for i in self._fresh(chunks)]
            if not fresh:
                return
            if any(c.embedding is None for c in fresh):
                raise ValueError("every chunk needs an embedding")
            emb = np.asarray([c.embedding for c in fresh], dtype=np.float32)
            if emb.ndim != 2:
                raise ValueError("embeddings must all have the same dimension")
            self._ensure_index(emb.shape[1])
            self._register(fresh, self._index.add(emb), emb)

    def add_chunks_device(self, chunks: list[Chunk], embeddings, stream: int | None = None) -> int:
        """add_chunks for embeddings that are already on the GPU (the in-process embedder's output):
        `embeddings` is a (len(chunks), dim) float32 device tensor; the vectors never visit the host
        on the index path (replaces embed_texts -> add_chunks, processors.py:413-418; a host copy is
        made only for the journal / keep_embeddings).  Returns the number added."""
        import torch

        if not chunks:
            return 0
        if embeddings.dim() != 2 or embeddings.shape[0] != len(chunks) or not embeddings.is_cuda:
            raise ValueError("embeddings must be a (len(chunks), dim) device tensor")
        with self._lock:
            keep = self._fresh(chunks)
            if not keep:
                return 0
            dev = embeddings.device
            # the given stream orders everything here: gathers / casts run on it too
            ctx = torch.cuda.stream(torch.cuda.ExternalStream(stream, device=dev)) if stream is not None \
                else contextlib.nullcontext()
            with ctx:
                emb = embeddings if len(keep) == len(chunks) else embeddings[torch.as_tensor(keep, device=dev)]
                emb = emb.to(torch.float32).contiguous()
                self._ensure_index(emb.shape[1])
                stream = torch.cuda.current_stream(dev).cuda_stream
                first = self._index.add_device(emb.data_ptr(), emb.shape[0], stream)
            need_host = self.keep_embeddings or (self.persist and not self._defer and self._gen > 0)
            self._register([chunks[i] for i in keep], first, emb.cpu().numpy() if need_host else None)
            return len(keep)

    def _remove_tables(self, rows: list[int], journal: bool = True) -> int:
        rows = [int(r) for r in rows if 0 <= r < len(self._records) and self._records[r] is not None]
        if not rows:
            return 0
        self._index.remove(np.asarray(rows, np.int64))
        for r in rows:
            rec = self._records[r]
            self._id_to_row.pop(rec[0], None)
            doc = self._doc_rows.get(rec[1])
            if doc is not None:
                doc.remove(r)
                if not doc:
                    del self._doc_rows[rec[1]]
            self._records[r] = None
            self._metas[r] = None
            self._live[r] = False
        if journal:
            self._log("del", rows=rows)
        return len(rows)

    def _delete_sync(self, chunk_ids: list[str]) -> None:
        with self._lock:
            if self._index is not None:
                self._remove_tables([self._id_to_row[c] for c in chunk_ids if c in self._id_to_row])

    async def delete(self, chunk_ids: list[str]) -> None:
        if not chunk_ids or self._index is None:
            return
        await asyncio.to_thread(self._delete_sync, chunk_ids)

    def _delete_document_sync(self, document_id: str) -> int:
        with self._lock:
            if self._index is None:
                return 0
            return self._remove_tables(list(self._doc_rows.get(document_id, ())))

    async def delete_by_document_id(self, document_id: str) -> int:
        if self._index is None or document_id not in self._doc_rows:  # (a new document: no thread hop)
            return 0
        n = await asyncio.to_thread(self._delete_document_sync, document_id)
        logger.info("deleted %d chunks for document_id %s", n, document_id)
        return n

    def _delete_by_metadata_sync(self, metadata_filter: dict[str, Any]) -> int:
        with self._lock:
            if self._index is None:
                return 0
            n = len(self._records)
            hit = F.evaluate(metadata_filter, self._cols) & self._live[:n]
            return self._remove_tables(np.nonzero(hit)[0].tolist())

    async def delete_by_metadata(self, metadata_filter: dict[str, Any]) -> int:
        if self._index is None or not metadata_filter:
            return 0
        return await asyncio.to_thread(self._delete_by_metadata_sync, metadata_filter)

    def _clear_sync(self):
        with self._lock:
            if self._journal is not None:
                self._journal.close()
            if self._index is not None:
                self._index.close()
            self._reset_tables()
            self._gen, self._journal = 0, None
            for p in self._paths.all_files():
                with contextlib.suppress(OSError):
                    os.remove(p)

    async def clear(self) -> None:
        await asyncio.to_thread(self._clear_sync)

    def delete_collection(self) -> None:
        """Drop the collection and its files (chroma_store.py:331, synchronous there too)."""
        self._clear_sync()

    def close(self) -> None:
        """Fold the journal into a snapshot and release the device index."""
        self._batcher.close()
        with self._lock:
            if self._journal is not None and self._journal.size:
                self.flush()
            if self._journal is not None:
                self._journal.close()
                self._journal = None
            if self._index is not None:
                self._index.close()
                self._index = None

    # ---------------------------------------------------------------- reads
    def _chunk(self, row: int, embedding=None, tables=None) -> Chunk:
        recs, metas = tables or (self._records, self._metas)
        rec = recs[row]
        meta = metas[row]
        # a fresh metadata dict per result, as Chroma returns (callers may mutate it)
        return Chunk(rec[0], meta.get("document_id", ""), rec[2], meta.get("chunk_index", 0), dict(meta),
                     embedding)

    def filter_bitmap(self, filters: dict[str, Any] | None):
        """uint64 row bitmap of a where-clause (None = no filter)."""
        if not filters:
            return None
        return F.evaluate_words(filters, self._cols)

    def _embeddings(self, rows: list[int]):
        if self.keep_embeddings and self._raw is not None:
            return self._raw[np.asarray(rows, np.int64)]
        return self._index.get_rows(rows)

    def search_batch(self, query_embeddings, top_k: int = 5, filters: dict[str, Any] | None = None
                     ) -> list[list[tuple[Chunk, float]]]:
        """Batched search: one GPU launch for all queries (BatchedVectorRetriever, the micro-batcher)."""
        prep = self._prep_search(query_embeddings, top_k, filters)
        return self._assemble(prep, self._run_search(prep))

    # search_batch in three steps, so the micro-batcher can run only the middle one in a worker thread
    # (it holds the GIL for little but the ctypes call; a worker doing the Python parts was starved by
    # a busy event loop) and assemble on the event-loop thread while the next launch runs
    def _prep_search(self, query_embeddings, top_k: int, filters):
        q = np.asarray(query_embeddings, dtype=np.float32)
        if q.ndim == 1:
            q = q[None, :]
        dim = self.dim
        if dim is not None and q.shape[1] != dim:
            raise ValueError(f"query dim {q.shape[1]} != collection dim {dim}")
        return (q, int(top_k), filters)

    def _run_search(self, prep):
        """The native search, under the store lock.  Everything that depends on the collection's
        current state -- the live row count, the filter bitmap (sized to the index's rows NOW, not when
        the query was queued: rows added in between would otherwise make the bitmap too short), the
        tables the rows resolve through -- is taken here, under the same lock as the search."""
        q, top_k, filters = prep
        with self._lock:  # ordered against mutations
            tables = (self._records, self._metas, self._epoch)
            n_live = self.count_sync()
            if self._index is None or n_live == 0 or top_k <= 0:
                return None, tables
            # top_k beyond the live rows returns them all (Chroma/FAISS); beyond HR_MAX_K the native
            # search takes its exhaustive exact path (same results, one corpus pass per query)
            return self._index.search(q, min(top_k, n_live), self.filter_bitmap(filters)), tables

    def search_device_sync(self, q, top_k: int):
        """(raw, tables) of an unfiltered search of the queries in `q`, a (B, dim) float32 torch tensor that may live
        on the GPU (the in-process embedder's output): the native search reads it in place and only the B * k results
        come back to the host -- no query vectors through host memory (the fused retrieve, retriever.py).  Pass the
        result with prep = (q, top_k, None) to _assemble.  An index without a device entry point (tests) gets a host
        copy."""
        import torch

        if q.dim() != 2 or (self.dim is not None and q.shape[1] != self.dim):
            raise ValueError(f"queries must be (B, {self.dim})")
        with self._lock:  # ordered against mutations, as _run_search
            tables = (self._records, self._metas, self._epoch)
            n_live = self.count_sync()
            idx = self._index
            if idx is None or n_live == 0 or top_k <= 0:
                return None, tables
            k = min(int(top_k), n_live)
            if (not q.is_cuda or not hasattr(idx, "search_device") or k > _native.HR_MAX_K
                    or len(getattr(idx, "devices", (0,))) > 1):
                return idx.search(q.detach().cpu().numpy(), k, None), tables
            q = q.to(torch.float32).contiguous()
            B = q.shape[0]
            ns = (B * k + 1) // 2 * 2  # scores, then the rows 8-byte aligned: one buffer, one copy back
            out = torch.empty((ns + 2 * B * k,), dtype=torch.float32, device=q.device)
            s_out, r_out = out[:B * k], out[ns:].view(torch.int64)
            st = torch.cuda.current_stream(q.device)
            idx.search_device(q.data_ptr(), B, k, s_out.data_ptr(), r_out.data_ptr(), stream=st.cuda_stream)
            host = out.cpu().numpy()  # (after the search, on the same stream)
            return (host[:B * k].reshape(B, k).copy(), host[ns:].view(np.int64).reshape(B, k).copy()), tables

    def _submit_native(self, prep, batcher: _SearchBatcher, loop):
        """Launch an unfiltered batch through the asynchronous native entry point from the event loop
        (None: this batch takes the worker-thread path -- a filter, no async-capable index, k beyond
        HR_MAX_K, an empty collection, or the store / handle busy: nothing here ever waits)."""
        q, top_k, filters = prep
        idx = self._index
        if (filters or idx is None or not self.native_async or top_k <= 0 or top_k > _native.HR_MAX_K
                or not hasattr(idx, "search_submit_host") or len(getattr(idx, "devices", (0,))) > 1):
            return None
        if not self._lock.acquire(blocking=False):  # a mutation (in a worker thread) holds the store
            return None
        try:
            n_live = self.count_sync()
            if n_live == 0 or self._index is not idx:
                return None
            fd = batcher.native_fd(loop)
            if fd < 0:
                return None
            k = min(top_k, n_live)
            try:
                ticket = idx.search_submit_host(q, k, fd)
            except (NotImplementedError, _native.BusyError):
                return None
            return idx, ticket, q.shape[0], k, (self._records, self._metas, self._epoch)
        finally:
            self._lock.release()

    def _collect_native(self, info, blocking: bool):
        """(raw, tables) of a finished native launch, as _run_search returns them; None when not blocking
        and the store lock is held, the handle is busy or the batch needs its exact fallback (the caller then
        collects in a worker thread)."""
        idx, ticket, B, k, tables = info
        if not self._lock.acquire(blocking=blocking):
            return None
        try:
            if idx is not self._index or tables[2] != self._epoch:  # cleared / closed since: rows are gone
                return None, tables
            if not blocking and hasattr(idx, "search_poll"):
                # a batch whose collect would run the exact fallback (a synchronous corpus pass) or a handle held
                # by another call: collect in a worker thread, never on the event loop
                try:
                    if idx.search_poll(ticket) != 1:
                        return None
                except _native.BusyError:
                    return None
            return idx.search_collect(ticket, B, k), tables
        finally:
            self._lock.release()

    def _gather(self, ran):
        """The host lists of a finished batch's hits -- (rec_l, meta_l, score_l, per_q, embs) -- or None when the store
        was cleared since the search ran (its rows are gone).  The hits' host records are gathered for the whole batch
        at once (object-array fancy indexing instead of a Python lookup per row and field)."""
        raw, (recs, metas, epoch) = ran
        if raw is None or epoch != self._epoch:
            return None
        scores, rows = raw
        # the tables the search ran against (append-only; a row deleted since then reads None, dropped)
        # rows the index returned but the tables do not hold yet (an add racing a native launch) are
        # treated like rows added after the search
        valid = (rows >= 0) & (rows < min(len(recs), len(metas)))
        hit_rows = rows[valid]
        rec_l = recs.a[hit_rows].tolist()
        meta_l = metas.a[hit_rows].tolist()
        score_l = scores[valid].tolist()
        per_q = valid.sum(axis=1).tolist()
        embs = None
        if self.include_embeddings and len(hit_rows):
            keep = [i for i, r in enumerate(rec_l) if r is not None]
            with self._lock:
                if epoch != self._epoch:
                    return None
                e = self._embeddings(hit_rows[keep].tolist())
            embs = [None] * len(rec_l)
            for j, i in enumerate(keep):
                embs[i] = e[j].tolist()
        return rec_l, meta_l, score_l, per_q, embs

    def _assemble(self, prep, ran) -> list[list[tuple[Chunk, float]]]:
        """(Chunk, score) lists of a finished batch.  Runs on the event loop while the next launch is in
        flight, so it is the host's per-hit cost under load: each hit is a slotted Chunk (two tracked objects per hit
        with its tuple) with a fresh metadata dict, as Chroma returns."""
        g = self._gather(ran)
        if g is None:
            return [[] for _ in range(len(prep[0]))]
        return (_hostfast.assemble if _hostfast is not None else _assemble_py)(Chunk, *g, self.untracked_results)

    def _assemble_results(self, ran, ks: list[int], ths: list[float], result_cls) -> list[list]:
        """A finished batch as the retriever's per-call results (result_cls(chunk, score, rank): top_k ks[q], threshold
        ths[q], ranks before the threshold -- base_retriever.py:66-80 without a reranker), built in one pass without
        the (Chunk, score) pairs: one tracked object fewer per hit for the cycle collector, and no Chunk for a hit past
        its call's top_k."""
        g = self._gather(ran)
        if g is None:
            return [[] for _ in ks]
        fn = _hostfast.assemble_results if _hostfast is not None else _assemble_results_py
        return fn(Chunk, result_cls, *g, [int(k) for k in ks], [float(t) for t in ths], self.untracked_results)

    async def search(self, query_embedding: list[float], top_k: int = 5, filters: dict[str, Any] | None = None
                     ) -> list[tuple[Chunk, float]]:
        if int(top_k) <= 0:
            return []
        q = np.asarray(query_embedding, dtype=np.float32).reshape(-1)
        return await self._batcher.submit(q, top_k, filters)

    def get_by_id_sync(self, chunk_id: str) -> Chunk | None:
        with self._lock:
            row = self._id_to_row.get(chunk_id)
            if row is None:
                return None
            return self._chunk(row, self._embeddings([row])[0].tolist())

    async def get_by_id(self, chunk_id: str) -> Chunk | None:
        return await asyncio.to_thread(self.get_by_id_sync, chunk_id)

    def count_sync(self) -> int:
        return len(self._id_to_row)

    async def count(self) -> int:
        return self.count_sync()


class VectorStoreFactory:
    """``VectorStoreFactory.create(config)`` like storage/base_storage.py:15-43.

    "hip" selects the MI355X index; "chroma" configs (the reference default) are
    served by the same index, which reproduces Chroma's add/query/where semantics
    with exact search (a persisted Chroma directory is not read)."""

    @staticmethod
    def create(config: VectorStoreConfig, **kwargs) -> BaseVectorStore:
        backend = config.backend.lower()
        if backend in ("hip", "chroma"):
            return HipVectorStore(config=config, **kwargs)
        raise ValueError(f"Unsupported vector store backend: {backend}")

    @staticmethod
    def list_backends() -> list[str]:
        return ["hip", "chroma"]

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
    ``filters`` are compiled to a row bitmap (plain dict or Chroma where-clause)
    and applied inside the scan, i.e. exact top-k among matching rows;
  * delete / delete_by_document_id / delete_by_metadata (chroma :150-222):
    row tombstones in the index + removal from the host tables;
  * get_by_id (chroma :224-247) returns the stored (normalised, quantised) vector
    as ``embedding``; count / clear / delete_collection.
Host tables (row -> chunk record, chunk id -> row) play the role of FAISS's
id_to_idx / idx_to_chunk (faiss_store.py:52-54, :112-121).  Persistence:
``<persist_directory>/<collection>.hri`` (the device index) + ``.rows.jsonl``.
"""
from __future__ import annotations

import contextlib
import json
import logging
import os
from typing import Any

import numpy as np

from .. import _native
from . import filters as F
from .base import BaseVectorStore, Chunk
from .config import VectorStoreConfig

logger = logging.getLogger(__name__)

_METRIC = {"cosine": "cosine", "dot": "ip", "euclidean": "l2"}


class HipVectorStore(BaseVectorStore):
    def __init__(self, config: VectorStoreConfig, *, index_factory=None):
        self.config = config
        params = dict(config.index_params or {})
        self.dtype = params.get("dtype", "bf16")
        self.device = int(params.get("device", 0))
        self.capacity = int(params.get("capacity", 0))
        self.include_embeddings = bool(params.get("include_embeddings", False))
        self.persist = bool(params.get("persist", True))
        self.metric = _METRIC[config.distance_metric]
        if self.dtype not in _native.DTYPES:
            raise ValueError(f"unknown index dtype {self.dtype!r}")
        self._factory = index_factory or (lambda dim: _native.NativeIndex(dim, self.dtype, self.metric, self.device))
        self._index = None
        self.dim: int | None = None
        self._records: list[dict | None] = []
        self._id_to_row: dict[str, int] = {}
        self._doc_rows: dict[str, list[int]] = {}
        self._cols = F.MetadataColumns()
        self._defer, self._dirty = 0, False
        if self.persist:
            self._load_if_present()

    # ---------------------------------------------------------------- persistence
    def _paths(self):
        base = os.path.join(self.config.persist_directory, self.config.collection_name)
        return base + ".hri", base + ".rows.jsonl"

    def _load_if_present(self):
        idx_path, rows_path = self._paths()
        if not (os.path.exists(idx_path) and os.path.exists(rows_path)):
            return
        with open(rows_path) as f:
            header = json.loads(f.readline())
            records = [json.loads(line) for line in f]
        self.dim = int(header["dim"])
        self._index = _native.NativeIndex.load(idx_path, device=self.device, dim=self.dim, dtype=header["dtype"],
                                               metric=header["metric"])
        self._records = records
        for row, rec in enumerate(records):
            if rec is not None:
                self._id_to_row[rec["id"]] = row
                self._doc_rows.setdefault(rec["document_id"], []).append(row)
        self._cols.append([(rec or {}).get("metadata", {}) for rec in records])
        logger.info("loaded %d chunks from %s", len(self._id_to_row), idx_path)

    @contextlib.contextmanager
    def deferred_save(self):
        """Write the persist files once at the end of a block of adds/deletes (bulk ingest)."""
        self._defer += 1
        try:
            yield self
        finally:
            self._defer -= 1
            if self._defer == 0 and self._dirty:
                self._save()

    def _save(self):
        if not self.persist or self._index is None:
            return
        if self._defer:
            self._dirty = True
            return
        self._dirty = False
        os.makedirs(self.config.persist_directory, exist_ok=True)
        idx_path, rows_path = self._paths()
        self._index.save(idx_path)
        tmp = rows_path + ".tmp"
        with open(tmp, "w") as f:
            f.write(json.dumps({"dim": self.dim, "dtype": self.dtype, "metric": self.metric}) + "\n")
            for rec in self._records:
                f.write(json.dumps(rec) + "\n")
        os.replace(tmp, rows_path)

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

    def _register(self, fresh: list[Chunk], first: int):
        metas = []
        for i, c in enumerate(fresh):
            meta = {"document_id": c.document_id, "chunk_index": c.chunk_index,
                    **{k: v for k, v in (c.metadata or {}).items() if v is not None}}
            rec = {"id": c.id, "document_id": c.document_id, "content": c.content, "chunk_index": c.chunk_index,
                   "metadata": meta}
            assert first + i == len(self._records)
            self._records.append(rec)
            self._id_to_row[c.id] = first + i
            self._doc_rows.setdefault(c.document_id, []).append(first + i)
            metas.append(meta)
        self._cols.append(metas)
        self._save()
        logger.info("added %d chunks to %s", len(fresh), self.config.collection_name)

    async def add_chunks(self, chunks: list[Chunk]) -> None:
        if not chunks:
            return
        fresh = [chunks[i] for i in self._fresh(chunks)]
        if not fresh:
            return
        if any(c.embedding is None for c in fresh):
            raise ValueError("every chunk needs an embedding")
        emb = np.asarray([c.embedding for c in fresh], dtype=np.float32)
        if emb.ndim != 2:
            raise ValueError("embeddings must all have the same dimension")
        self._ensure_index(emb.shape[1])
        self._register(fresh, self._index.add(emb))

    def add_chunks_device(self, chunks: list[Chunk], embeddings, stream: int | None = None) -> int:
        """add_chunks for embeddings that are already on the GPU (the in-process embedder's output):
        `embeddings` is a (len(chunks), dim) float32 device tensor; the vectors never visit the host
        (replaces embed_texts -> add_chunks, processors.py:413-418).  Returns the number added."""
        import torch

        if not chunks:
            return 0
        if embeddings.dim() != 2 or embeddings.shape[0] != len(chunks) or not embeddings.is_cuda:
            raise ValueError("embeddings must be a (len(chunks), dim) device tensor")
        keep = self._fresh(chunks)
        if not keep:
            return 0
        emb = embeddings if len(keep) == len(chunks) else embeddings[torch.as_tensor(keep, device=embeddings.device)]
        emb = emb.to(torch.float32).contiguous()
        self._ensure_index(emb.shape[1])
        if stream is None:
            stream = torch.cuda.current_stream(emb.device).cuda_stream
        first = self._index.add_device(emb.data_ptr(), emb.shape[0], stream)
        self._register([chunks[i] for i in keep], first)
        return len(keep)

    def _remove_rows(self, rows: list[int]) -> int:
        rows = [r for r in rows if self._records[r] is not None]
        if not rows:
            return 0
        self._index.remove(np.asarray(rows, np.int64))
        for r in rows:
            rec = self._records[r]
            self._id_to_row.pop(rec["id"], None)
            doc = self._doc_rows.get(rec["document_id"])
            if doc is not None:
                doc.remove(r)
                if not doc:
                    del self._doc_rows[rec["document_id"]]
            self._records[r] = None
        self._save()
        return len(rows)

    async def delete(self, chunk_ids: list[str]) -> None:
        if not chunk_ids or self._index is None:
            return
        self._remove_rows([self._id_to_row[c] for c in chunk_ids if c in self._id_to_row])

    async def delete_by_document_id(self, document_id: str) -> int:
        if self._index is None:
            return 0
        n = self._remove_rows(list(self._doc_rows.get(document_id, ())))
        logger.info("deleted %d chunks for document_id %s", n, document_id)
        return n

    async def delete_by_metadata(self, metadata_filter: dict[str, Any]) -> int:
        if self._index is None or not metadata_filter:
            return 0
        hit = F.evaluate(metadata_filter, self._cols) & self._live_mask()
        return self._remove_rows(np.nonzero(hit)[0].tolist())

    def _clear_sync(self):
        if self._index is not None:
            self._index.close()
        self._index, self.dim = None, None
        self._records, self._id_to_row, self._doc_rows = [], {}, {}
        self._cols.clear()
        for p in self._paths():
            if os.path.exists(p):
                os.remove(p)

    async def clear(self) -> None:
        self._clear_sync()

    def delete_collection(self) -> None:
        """Drop the collection and its files (chroma_store.py:331, synchronous there too)."""
        self._clear_sync()

    # ---------------------------------------------------------------- reads
    def _live_mask(self) -> np.ndarray:
        return np.array([rec is not None for rec in self._records], dtype=bool)

    def _chunk(self, row: int, embedding=None) -> Chunk:
        rec = self._records[row]
        meta = rec["metadata"]
        return Chunk(id=rec["id"], document_id=meta.get("document_id", ""), content=rec["content"],
                     chunk_index=meta.get("chunk_index", 0), metadata=dict(meta), embedding=embedding)

    def _filter_bitmap(self, filters: dict[str, Any] | None):
        if not filters:
            return None
        return F.to_bitmap(F.evaluate(filters, self._cols))

    def search_batch(self, query_embeddings, top_k: int = 5, filters: dict[str, Any] | None = None
                     ) -> list[list[tuple[Chunk, float]]]:
        """Batched search: one GPU launch for all queries (used by BatchedVectorRetriever)."""
        q = np.asarray(query_embeddings, dtype=np.float32)
        if q.ndim == 1:
            q = q[None, :]
        if self._index is None or self.count_sync() == 0:
            return [[] for _ in range(len(q))]
        if q.shape[1] != self.dim:
            raise ValueError(f"query dim {q.shape[1]} != collection dim {self.dim}")
        # top_k beyond the live rows returns them all (Chroma/FAISS); beyond HR_MAX_K the native
        # search takes its exhaustive exact path (same results, one corpus pass per query)
        if int(top_k) <= 0:
            return [[] for _ in range(len(q))]
        k = min(int(top_k), self.count_sync())
        scores, rows = self._index.search(q, k, self._filter_bitmap(filters))
        out = []
        for b in range(len(q)):
            valid = [(int(r), float(s)) for r, s in zip(rows[b], scores[b]) if r >= 0]
            embs = None
            if self.include_embeddings and valid:
                embs = self._index.get_rows([r for r, _ in valid])
            out.append([(self._chunk(r, None if embs is None else embs[i].tolist()), s)
                        for i, (r, s) in enumerate(valid)])
        return out

    async def search(self, query_embedding: list[float], top_k: int = 5, filters: dict[str, Any] | None = None
                     ) -> list[tuple[Chunk, float]]:
        return self.search_batch([query_embedding], top_k, filters)[0]

    async def get_by_id(self, chunk_id: str) -> Chunk | None:
        row = self._id_to_row.get(chunk_id)
        if row is None:
            return None
        return self._chunk(row, self._index.get_rows([row])[0].tolist())

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

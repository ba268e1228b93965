"""KB ingest slice on one GPU: split -> embed (in-process) -> add to the HIP index (config 4).

Restates BaseProcessor._chunk_and_store (utu/rag/knowledge_builder/processors.py:340-421):
for each document, old chunks with the same document_id are deleted first (:363-369),
the text is split with the configured RecursiveTextSplitter (:385), chunk i gets
id f"{document.id}_chunk_{i}", document metadata without "_"-prefixed keys plus
index_type="index_content" unless present, updated with the call's extra metadata
(:387-407), and the chunk texts are embedded and added to the store (:412-418).

What changes is where the vectors go: with the in-process TorchRocmEmbedder, texts of
many documents are packed into full embedder batches and each batch's (B, H) float32
device tensor is appended to the index by hr_index_add_device -- the embeddings never
visit the host.  Any other BaseEmbedder (host lists) falls back to add_chunks.
After a document's chunks, its summary vector is added as the reference's simple-document
processor does (processors.py:559-561 -> _create_summary_index :423-464): one chunk
``f"{doc}_summary"`` with content ``f"{source or doc id}\n{summary}"``, chunk_index -1 and the
document's whole metadata (``_``-keys included, as the reference stores them) plus
index_type="index_summary" -- the vectors kb_file_search searches (kb_search_toolkit.py:530-535).
Documents flagged ``_use_hierarchical_splitter`` (chunklevel.md, processors.py:226-332) are split by
HierarchicalMarkdownSplitter with the configured chunk size and overlap (processors.py:371-379).
"""
from __future__ import annotations

import logging
from typing import Any

from .base import BaseEmbedder, Chunk, Document
from .chunker import HierarchicalMarkdownSplitter, RecursiveTextSplitter
from .config import ChunkingConfig

logger = logging.getLogger(__name__)


def summary_chunk(document: Document) -> Chunk:
    """The document's summary-index record (processors.py:423-464)."""
    meta = document.metadata or {}
    content = f"{meta.get('source', document.id)}\n{meta.get('summary') or ''}"
    return Chunk(id=f"{document.id}_summary", document_id=document.id, content=content, chunk_index=-1,
                 metadata={**meta, "index_type": "index_summary"})


def make_chunks(document: Document, texts: list[str], metadata: dict[str, Any] | None = None) -> list[Chunk]:
    """Chunk records of one document exactly as processors.py:387-407 builds them."""
    chunks = []
    for i, text in enumerate(texts):
        meta = {k: v for k, v in (document.metadata or {}).items() if not k.startswith("_")}
        meta.setdefault("index_type", "index_content")
        chunks.append(Chunk(id=f"{document.id}_chunk_{i}", document_id=document.id, content=text, chunk_index=i,
                            metadata=meta))
    if metadata:
        for c in chunks:
            c.metadata.update(metadata)
    return chunks


class GpuIngestor:
    """split -> embed -> add for a HipVectorStore, batching embedder work across documents."""

    def __init__(self, vector_store, embedder: BaseEmbedder, chunker=None, chunking: ChunkingConfig | None = None,
                 embed_batch: int | None = None, summary_index: bool = True, pack_batches: int = 16):
        self.vector_store = vector_store
        self.summary_index = bool(summary_index)
        self.embedder = embedder
        self.chunker = chunker or RecursiveTextSplitter(chunking or ChunkingConfig())
        self.embed_batch = int(embed_batch or getattr(embedder, "batch_size", 64))
        self._device = hasattr(embedder, "embed_texts_device") and hasattr(vector_store, "add_chunks_device")
        # chunks handed to the in-process embedder at once: it length-sorts a pack into its batches, so
        # each batch pads to about its own length instead of the longest of a random mix (one batch per
        # pack: 32 % of the forward's token positions were padding at 500-character chunks)
        if self._device:
            self.embed_batch *= max(1, int(pack_batches))
        # device path, pipelined one batch deep: batch i's vectors are added while batch i+1's forward
        # runs -- (chunks, vectors, ready event) of the batch embedded but not yet added
        self._inflight = None
        self._add_stream = None

    def split(self, document: Document, metadata: dict[str, Any] | None = None) -> list[Chunk]:
        chunker = self.chunker
        if (document.metadata or {}).get("_use_hierarchical_splitter", False):
            cfg = getattr(self.chunker, "config", None) or ChunkingConfig()
            chunker = HierarchicalMarkdownSplitter(ChunkingConfig(strategy="hierarchical", chunk_size=cfg.chunk_size,
                                                                  chunk_overlap=cfg.chunk_overlap))
        return make_chunks(document, chunker.split_text(document.content, document.metadata), metadata)

    def _flush(self) -> int:
        """Add the batch embedded last (its vectors on the device), ordered after its own forward only:
        the add stream waits for that batch's event, not for the forward enqueued after it."""
        if self._inflight is None:
            return 0
        chunks, emb, ready, _ = self._inflight
        self._inflight = None
        self._add_stream.wait_event(ready)
        return self.vector_store.add_chunks_device(chunks, emb, stream=self._add_stream.cuda_stream)

    async def _store(self, chunks: list[Chunk]) -> int:
        if not chunks:
            return 0
        texts = [c.content for c in chunks]
        if self._device:
            import torch

            if self._add_stream is None:
                self._add_stream = torch.cuda.Stream(getattr(self.embedder, "device", None))
            emb = self.embedder.embed_texts_device(texts)  # enqueued; the host goes on at once
            ready = torch.cuda.Event()
            ready.record(torch.cuda.current_stream(emb.device))
            n = self._flush()  # the previous batch, while this forward runs
            self._inflight = (chunks, emb, ready, {c.document_id for c in chunks})
            return n
        for c, e in zip(chunks, await self.embedder.embed_texts(texts)):
            c.embedding = e
        await self.vector_store.add_chunks(chunks)
        return len(chunks)

    async def chunk_and_store(self, document: Document, metadata: dict[str, Any] | None = None) -> int:
        """One document (BaseProcessor._chunk_and_store).  Returns the number of chunks created."""
        return await self.ingest([document], metadata)

    async def ingest(self, documents: list[Document], metadata: dict[str, Any] | None = None) -> int:
        """Many documents; embedder batches span document boundaries.  Returns chunks created."""
        created, pending, pending_docs = 0, [], set()
        try:
            with self.vector_store.deferred_save():
                for doc in documents:
                    if doc.id in pending_docs or (self._inflight is not None and doc.id in self._inflight[3]):
                        # same id twice: store the first copy first
                        await self._store(pending)
                        self._flush()
                        pending, pending_docs = [], set()
                    created += await self._one(doc, metadata, pending)
                    pending_docs.add(doc.id)
                    if len(pending) >= self.embed_batch:
                        while len(pending) >= self.embed_batch:
                            await self._store(pending[:self.embed_batch])
                            pending = pending[self.embed_batch:]
                        pending_docs = {c.document_id for c in pending}
                await self._store(pending)
                self._flush()
        except BaseException:
            # a failed ingest commits nothing later: drop the embedded batch still in flight (the next call
            # would otherwise store it silently, after newer data)
            self._inflight = None
            raise
        return created

    async def _one(self, doc: Document, metadata, pending: list[Chunk]) -> int:
        try:
            n_old = await self.vector_store.delete_by_document_id(doc.id)
            if n_old:
                logger.info("deleted %d old chunks for document %s", n_old, doc.id)
        except Exception as e:  # the reference carries on (processors.py:367-369)
            logger.warning("failed to delete old chunks for %s: %s", doc.id, e)
        chunks = self.split(doc, metadata)
        if not chunks:
            logger.warning("no chunks created for document %s", doc.id)
        pending.extend(chunks)
        if self.summary_index:  # created even when the document gave no chunks (processors.py:559-561)
            pending.append(summary_chunk(doc))
        return len(chunks)

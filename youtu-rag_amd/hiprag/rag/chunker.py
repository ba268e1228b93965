"""RecursiveTextSplitter with the reference's exact output (ingest slice, config C4).

Behaviour of utu/rag/knowledge_builder/chunker.py:10-121, including its quirks:
separators tried in order ["\\n\\n", "\\n", ". ", " ", ""]; pieces are packed
greedily while the running chunk stays <= chunk_size characters (the separator
is kept on every piece but the last when keep_separator); an oversized piece is
split recursively with the remaining separators; the fixed-length fallback
steps by chunk_size - chunk_overlap; overlap then PREPENDS the previous chunk's
last chunk_overlap characters to every chunk after the first (so chunks may
exceed chunk_size); chunks are stripped and empty ones dropped.  Pinned by
tests/golden/chunker.json (produced by the reference splitter itself).
"""
from __future__ import annotations

from typing import Any

from .base import BaseTextSplitter
from .config import ChunkingConfig

DEFAULT_SEPARATORS = ["\n\n", "\n", ". ", " ", ""]


class RecursiveTextSplitter(BaseTextSplitter):
    def __init__(self, config: ChunkingConfig | None = None):
        self.config = config or ChunkingConfig(strategy="recursive")
        self.separators = self.config.separators or list(DEFAULT_SEPARATORS)

    def split_text(self, text: str, metadata: dict[str, Any] | None = None) -> list[str]:
        return self._split(text, self.separators)

    def _split(self, text: str, seps: list[str]) -> list[str]:
        size, keep = self.config.chunk_size, self.config.keep_separator
        if not seps or seps[0] == "":
            return self._by_length(text)
        sep, rest = seps[0], seps[1:]
        parts = text.split(sep)
        last = len(parts) - 1
        chunks: list[str] = []
        cur = ""
        for i, part in enumerate(parts):
            tail = sep if keep and i < last else ""
            if len(cur + part + tail) <= size:
                cur = cur + part + tail
                continue
            if cur:
                chunks.append(cur)
            if len(part) > size:
                chunks.extend(self._split(part, rest))
                cur = ""
            else:
                cur = part + tail
        if cur:
            chunks.append(cur)
        if self.config.chunk_overlap > 0 and len(chunks) > 1:
            ov = self.config.chunk_overlap
            chunks = [chunks[0]] + [chunks[i - 1][-ov:] + chunks[i] for i in range(1, len(chunks))]
        return [c.strip() for c in chunks if c.strip()]

    def _by_length(self, text: str) -> list[str]:
        size, step = self.config.chunk_size, self.config.chunk_size - self.config.chunk_overlap
        return [text[i:i + size] for i in range(0, len(text), step)]

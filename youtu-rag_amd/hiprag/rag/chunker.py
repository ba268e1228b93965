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

import re
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


_H1 = re.compile(r"^#\s+(.+)$")
_H2 = re.compile(r"^##\s+(.+)$")


class HierarchicalMarkdownSplitter(BaseTextSplitter):
    """Heading-aware splitter for ``*_chunklevel.md`` documents (utu/rag/knowledge_builder/chunker.py:124-349).

    A line ``# t`` opens a new H1 section (and closes any H2), ``## t`` a new H2 section; other
    non-blank lines are content, kept whole.  Sections without content produce nothing.  Each section
    is packed greedily by whole lines: a line (+1 for its newline) joins the current chunk while the
    header length + the chunk's line lengths stay <= chunk_size; every chunk carries the header block
    ``# h1\\n## h2`` followed by a blank line.  With chunk_overlap, chunk i > 0 of a section gets the
    last chunk_overlap characters of chunk i-1's body (left-stripped) on a line of its own after the
    header.  Chunks are stripped, empty ones dropped.  Pinned by tests/golden/hierarchical.json.
    """

    def __init__(self, config: ChunkingConfig | None = None):
        self.config = config or ChunkingConfig(strategy="hierarchical")

    def split_text(self, text: str, metadata: dict[str, Any] | None = None) -> list[str]:
        if not text or not text.strip():
            return []
        out: list[str] = []
        for h1, h2, lines in self._sections(text):
            out.extend(self._pack(h1, h2, lines))
        return [c.strip() for c in out if c.strip()]

    @staticmethod
    def _sections(text: str):
        """(h1, h2, content lines) per section that has content, in document order."""
        h1 = h2 = None
        lines: list[str] = []
        for line in text.split("\n"):
            m1 = _H1.match(line)
            m2 = None if m1 else _H2.match(line)
            if m1 or m2:
                if lines:
                    yield h1, h2, lines
                    lines = []
                if m1:
                    h1, h2 = m1.group(1).strip(), None
                else:
                    h2 = m2.group(1).strip()
            elif line.strip():
                lines.append(line)
        if lines:
            yield h1, h2, lines

    def _pack(self, h1, h2, lines: list[str]) -> list[str]:
        header = "\n".join(([f"# {h1}"] if h1 else []) + ([f"## {h2}"] if h2 else []))
        size = self.config.chunk_size
        bodies: list[list[str]] = []
        cur: list[str] = []
        used = len(header)
        for line in lines:
            need = len(line) + 1
            if cur and used + need > size:
                bodies.append(cur)
                cur, used = [], len(header)
            cur.append(line)
            used += need
        if cur:
            bodies.append(cur)
        texts = ["\n".join(b) for b in bodies]
        wrap = (lambda body: f"{header}\n\n{body}") if header else (lambda body: body)
        ov = self.config.chunk_overlap
        if ov <= 0 or len(texts) < 2:
            return [wrap(t) for t in texts]
        # the body of a wrapped chunk is what follows the header with its leading newlines removed,
        # i.e. the joined lines with any leading newline characters dropped
        strip_nl = (lambda t: t.lstrip("\n")) if header else (lambda t: t)
        out = [wrap(texts[0])]
        for prev, body in zip(texts, texts[1:]):
            out.append(wrap(f"{strip_nl(prev)[-ov:].lstrip()}\n{strip_nl(body)}"))
        return out

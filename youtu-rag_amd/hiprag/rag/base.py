"""Plugin interfaces of the KB-search path, re-declared for drop-in use.

Names, fields and method signatures match utu/rag/base.py of the reference
(Document :12, Chunk :26, RetrievalResult :42, QueryRequest/QueryResponse :54/:64,
BuildStatus :74, HealthStatus :87, BaseTextSplitter :104, BaseEmbedder :113,
BaseReranker :127, BaseKnowledgeBuilder :150, BaseRetriever :171,
BaseVectorStore :187, BaseStorageMonitor :235), so code written against the
reference's ABCs runs unchanged against hiprag's implementations.  All
data-plane methods stay ``async``, as in the reference.
"""
from __future__ import annotations

from abc import ABC, abstractmethod
from dataclasses import dataclass
from typing import Any

from pydantic import BaseModel, Field


def _preview(text: str, n: int = 50) -> str:
    return text[:n] + "..." if len(text) > n else text


@dataclass
class Document:
    id: str
    content: str
    metadata: dict[str, Any] | None = None
    embedding: list[float] | None = None

    def __repr__(self) -> str:
        return f"Document(id={self.id}, content='{_preview(self.content)}', metadata={self.metadata})"


# Chunk and RetrievalResult carry __slots__ (the reference's are plain dataclasses, same fields and order): a search
# returns one of each per hit, and without a per-instance __dict__ each hit is one tracked object fewer for Python's
# cycle collector to promote and walk under load (tools/bench_store_host.py)
@dataclass(slots=True)
class Chunk:
    id: str
    document_id: str
    content: str
    chunk_index: int
    metadata: dict[str, Any] | None = None
    embedding: list[float] | None = None

    def __repr__(self) -> str:
        return (f"Chunk(id={self.id}, doc_id={self.document_id}, index={self.chunk_index}, "
                f"content='{_preview(self.content)}')")


@dataclass(slots=True)
class RetrievalResult:
    chunk: Chunk
    score: float
    rank: int | None = None

    def __repr__(self) -> str:
        return f"RetrievalResult(chunk_id={self.chunk.id}, score={self.score:.4f}, rank={self.rank})"


class QueryRequest(BaseModel):
    query: str
    top_k: int = 5
    filters: dict[str, Any] | None = None
    enable_reranking: bool = False
    similarity_threshold: float | None = None


class QueryResponse(BaseModel):
    query: str
    results: list[dict[str, Any]]
    total_results: int
    retrieval_time_ms: float
    metadata: dict[str, Any] = Field(default_factory=dict)


class _RecordModel(BaseModel):
    """Field helpers the reference gets from utu/db/utu_basemodel.py."""

    def update(self, **kwargs):
        for key, value in kwargs.items():
            if hasattr(self, key):
                setattr(self, key, value)

    def get(self, key, default=None):
        return getattr(self, key, default)

    @classmethod
    def from_dict(cls, data: dict):
        return cls(**data)

    def as_dict(self) -> dict:
        return {k: v for k, v in self.model_dump().items() if v is not None}


class BuildStatus(_RecordModel):
    status: str
    total_documents: int = 0
    processed_documents: int = 0
    total_chunks: int = 0
    errors: list[str] = Field(default_factory=list)
    start_time: str | None = None
    end_time: str | None = None
    metadata: dict[str, Any] = Field(default_factory=dict)


class HealthStatus(_RecordModel):
    is_healthy: bool
    backend: str
    collection_name: str
    total_documents: int = 0
    total_chunks: int = 0
    index_size_bytes: int = 0
    last_check_time: str
    errors: list[str] = Field(default_factory=list)
    warnings: list[str] = Field(default_factory=list)
    metadata: dict[str, Any] = Field(default_factory=dict)


class BaseTextSplitter(ABC):
    @abstractmethod
    def split_text(self, text: str, metadata: dict[str, Any] | None = None) -> list[str]:
        """Split ``text`` into chunk strings."""


class BaseEmbedder(ABC):
    @abstractmethod
    async def embed_texts(self, texts: list[str]) -> list[list[float]]:
        """Passage embeddings, one vector per text."""

    @abstractmethod
    async def embed_query(self, query: str) -> list[float]:
        """Query embedding."""


class BaseReranker(ABC):
    @abstractmethod
    async def rerank(self, query: str, results: list[RetrievalResult], top_k: int | None = None
                     ) -> list[RetrievalResult]:
        """Re-order ``results`` by relevance to ``query`` (None: keep all)."""


class BaseKnowledgeBuilder(ABC):
    @abstractmethod
    async def build_from_documents(self, documents: list[Document], rebuild: bool = False) -> BuildStatus:
        ...

    @abstractmethod
    async def add_documents(self, documents: list[Document]) -> BuildStatus:
        ...

    @abstractmethod
    async def get_build_status(self) -> BuildStatus:
        ...


class BaseRetriever(ABC):
    @abstractmethod
    async def retrieve(self, query: str, top_k: int = 5, **kwargs) -> list[RetrievalResult]:
        ...

    @abstractmethod
    async def batch_retrieve(self, queries: list[str], top_k: int = 5, **kwargs) -> list[list[RetrievalResult]]:
        ...


class BaseVectorStore(ABC):
    @abstractmethod
    async def add_chunks(self, chunks: list[Chunk]) -> None:
        ...

    @abstractmethod
    async def search(self, query_embedding: list[float], top_k: int = 5, filters: dict[str, Any] | None = None
                     ) -> list[tuple[Chunk, float]]:
        ...

    @abstractmethod
    async def delete(self, chunk_ids: list[str]) -> None:
        ...

    @abstractmethod
    async def delete_by_document_id(self, document_id: str) -> int:
        """Delete every chunk of ``document_id``; returns how many were deleted."""

    @abstractmethod
    async def get_by_id(self, chunk_id: str) -> Chunk | None:
        ...

    @abstractmethod
    async def count(self) -> int:
        ...

    @abstractmethod
    async def clear(self) -> None:
        ...


class BaseStorageMonitor(ABC):
    @abstractmethod
    async def check_health(self) -> HealthStatus:
        ...

    @abstractmethod
    async def collect_metrics(self) -> dict[str, Any]:
        ...

    @abstractmethod
    async def log_query(self, query: str, latency_ms: float, result_count: int) -> None:
        ...

    @abstractmethod
    async def get_query_stats(self, time_range_hours: int = 24) -> dict[str, Any]:
        ...

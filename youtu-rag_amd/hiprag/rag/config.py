"""Config surface of the KB-search path (pydantic), shaped like utu/rag/config.py.

Same class and field names and defaults as the reference (ChunkingConfig :10,
EmbeddingConfig :20, KnowledgeBuilderConfig :31, RetrieverConfig :42,
VectorStoreConfig :52, MonitorConfig :68, RAGConfig :85) so existing YAML
(configs/rag/*.yaml) validates unchanged.  Additions, all optional:
  * VectorStoreConfig.backend also accepts "hip" (the MI355X index); "chroma"
    configs are served by the same index (see storage.VectorStoreFactory);
  * VectorStoreConfig.index_params keys for the HIP index: dtype (bf16|f16|f32),
    device (int), capacity (rows), include_embeddings (bool), persist (bool);
  * EmbeddingConfig.provider also accepts "rocm" (the in-process embedder).
Secrets (api_key, base_url) are masked in repr like utu/config/base_config.py:22-38.
"""
from __future__ import annotations

from typing import Any, Literal

from pydantic import BaseModel, Field

_SECRET_KEYS = ("api_key", "base_url")


class ConfigBaseModel(BaseModel):
    def __repr__(self) -> str:
        parts = []
        for k, v in self.__repr_args__():
            hidden = k is not None and any(s in k.lower() for s in _SECRET_KEYS)
            parts.append(f"{k}={'***' if hidden else repr(v)}")
        return f"{self.__class__.__name__}({', '.join(parts)})"

    __str__ = __repr__

    def model_dump(self, *, exclude_none: bool = True, **kwargs) -> dict[str, Any]:
        return super().model_dump(exclude_none=exclude_none, **kwargs)


class ChunkingConfig(ConfigBaseModel):
    strategy: Literal["recursive", "hierarchical"] = "recursive"
    chunk_size: int = Field(default=1000, ge=100, le=10000)
    chunk_overlap: int = Field(default=200, ge=0, le=1000)
    separators: list[str] | None = None
    keep_separator: bool = True


class EmbeddingConfig(ConfigBaseModel):
    model: str = "text-embedding-3-small"
    provider: Literal["openai", "local", "huggingface", "rocm"] = "openai"
    api_key: str | None = None
    base_url: str | None = None
    batch_size: int = Field(default=32, ge=1, le=512)
    dimensions: int | None = None


class KnowledgeBuilderConfig(ConfigBaseModel):
    chunking: ChunkingConfig = Field(default_factory=ChunkingConfig)
    embedding: EmbeddingConfig = Field(default_factory=EmbeddingConfig)
    max_workers: int = Field(default=4, ge=1, le=16)
    enable_metadata: bool = True
    metadata_fields: list[str] = Field(default_factory=lambda: ["source", "page", "title"])
    batch_delay: float = Field(default=3.0, ge=0.0, le=60.0)


class RetrieverConfig(ConfigBaseModel):
    top_k: int = Field(default=5, ge=1)
    similarity_threshold: float = Field(default=0.7, ge=0.0, le=1.0)
    enable_reranking: bool = False
    reranker_model: str | None = None
    reranker_top_k: int = Field(default=3, ge=1, le=50)


class VectorStoreConfig(ConfigBaseModel):
    backend: Literal["chroma", "hip"] = "chroma"
    collection_name: str = "knowledge_base"
    persist_directory: str = "./data/vector_store"
    host: str | None = None
    port: int | None = None
    api_key: str | None = None
    distance_metric: Literal["cosine", "euclidean", "dot"] = "cosine"
    index_type: str | None = None
    index_params: dict[str, Any] = Field(default_factory=dict)


class MonitorConfig(ConfigBaseModel):
    enable_monitoring: bool = True
    health_check_interval: int = Field(default=60, ge=10, le=3600)
    metrics_retention_days: int = Field(default=30, ge=1, le=365)
    enable_query_logging: bool = True
    enable_alerts: bool = True
    alert_thresholds: dict[str, float] = Field(
        default_factory=lambda: {"query_latency_ms": 1000.0, "error_rate": 0.05, "index_size_gb": 100.0})


class RAGConfig(ConfigBaseModel):
    name: str = "default_rag"
    description: str | None = None
    knowledge_builder: KnowledgeBuilderConfig = Field(default_factory=KnowledgeBuilderConfig)
    retriever: RetrieverConfig = Field(default_factory=RetrieverConfig)
    vector_store: VectorStoreConfig = Field(default_factory=VectorStoreConfig)
    monitor: MonitorConfig = Field(default_factory=MonitorConfig)
    enable_cache: bool = True
    cache_ttl: int = Field(default=3600, ge=60, le=86400)
    log_level: Literal["DEBUG", "INFO", "WARNING", "ERROR"] = "INFO"

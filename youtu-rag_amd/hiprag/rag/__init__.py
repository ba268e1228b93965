"""Drop-in mirror of the reference's KB-search plugin API (utu/rag) backed by the MI355X index."""
from .base import (BaseEmbedder, BaseKnowledgeBuilder, BaseReranker, BaseRetriever, BaseStorageMonitor,
                   BaseTextSplitter, BaseVectorStore, BuildStatus, Chunk, Document, HealthStatus, QueryRequest,
                   QueryResponse, RetrievalResult)
from .builder import CourseSearcher, KnowledgeBuilder
from .chunker import HierarchicalMarkdownSplitter, RecursiveTextSplitter
from .config import (ChunkingConfig, EmbeddingConfig, KnowledgeBuilderConfig, MonitorConfig, RAGConfig,
                     RetrieverConfig, VectorStoreConfig)
from .embeddings import EmbedderFactory, ServiceEmbedder, create_embedder
from .rerankers import RerankerFactory, TorchRocmReranker
from .retriever import BatchedVectorRetriever, HybridRetriever, VectorRetriever
from .storage import HipVectorStore, VectorStoreFactory

__all__ = [
    "BaseEmbedder", "BaseKnowledgeBuilder", "BaseReranker", "BaseRetriever", "BaseStorageMonitor", "BaseTextSplitter",
    "BaseVectorStore", "BuildStatus", "Chunk", "Document", "HealthStatus", "QueryRequest", "QueryResponse",
    "RetrievalResult", "RecursiveTextSplitter", "HierarchicalMarkdownSplitter", "ChunkingConfig", "EmbeddingConfig", "KnowledgeBuilderConfig",
    "MonitorConfig", "RAGConfig", "RetrieverConfig", "VectorStoreConfig", "EmbedderFactory", "ServiceEmbedder",
    "create_embedder", "BatchedVectorRetriever", "HybridRetriever", "VectorRetriever", "HipVectorStore",
    "VectorStoreFactory", "RerankerFactory", "TorchRocmReranker", "KnowledgeBuilder", "CourseSearcher",
]

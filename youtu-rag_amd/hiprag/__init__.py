"""hiprag -- MI355X-native embedding + retrieval engine for youtu-rag's KB-search hot path.

``hiprag.rag`` re-declares the reference's plugin API (utu/rag/base.py, utu/rag/config.py)
and provides the HIP-backed implementations; ``hiprag._native`` binds libhiprag.so.
"""
__version__ = "0.1.0"

"""Deterministic text -> vector embedder for the caller fixtures (gen_builder.py and the tests that replay
them): each text's vector is a seeded Gaussian keyed by crc32(text).  Texts containing "POISON" make
embed_texts raise, to exercise the callers' per-document error handling."""
from __future__ import annotations

import zlib

import numpy as np

DIM = 48


def vec(text: str, dim: int = DIM) -> np.ndarray:
    return np.random.default_rng(zlib.crc32(text.encode("utf-8"))).standard_normal(dim).astype(np.float32)


class HashEmbedder:
    def __init__(self, dim: int = DIM, batch_size: int = 16):
        self.dim = dim
        self.batch_size = batch_size
        self.calls: list[int] = []  # sizes of the embed_texts calls

    async def embed_texts(self, texts):
        self.calls.append(len(texts))
        if any("POISON" in t for t in texts):
            raise ValueError("embedding service rejected a poisoned text")
        return [vec(t, self.dim).tolist() for t in texts]

    async def embed_query(self, query):
        return vec("query: " + query, self.dim).tolist()

    async def embed_queries(self, queries):
        return [vec("query: " + q, self.dim).tolist() for q in queries]

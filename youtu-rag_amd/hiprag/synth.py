"""Synthetic corpora and planted queries for benchmarks and tests.

The corpus generator is counter-based and keyed by the GLOBAL row index, so any
shard can produce its rows independently and the corpus is identical for every
GPU count.  Element (row, d) = sum of the four 16-bit
fields of splitmix64(seed*K + row*dim + d) minus 131070 -- an integer, exact in
fp32 -- the same recipe libhiprag.so's hr_index_add_synthetic runs on the device.
"""
from __future__ import annotations

import numpy as np

_MASK64 = (1 << 64) - 1


def _mix64(z: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = z + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def corpus_rows(seed: int, rows: np.ndarray, dim: int) -> np.ndarray:
    """Raw (un-normalised) fp32 rows for the given global row indices."""
    r = np.asarray(rows, np.uint64).reshape(-1, 1)
    d = np.arange(dim, dtype=np.uint64)[None, :]
    with np.errstate(over="ignore"):
        key = np.uint64((seed * 0xD1B54A32D192ED03) & _MASK64) + r * np.uint64(dim) + d
    z = _mix64(key)
    m = np.uint64(0xFFFF)
    v = ((z & m).astype(np.int64) + ((z >> np.uint64(16)) & m).astype(np.int64)
         + ((z >> np.uint64(32)) & m).astype(np.int64) + (z >> np.uint64(48)).astype(np.int64) - 131070)
    return v.astype(np.float32)


def planted_queries(seed: int, n_rows: int, dim: int, B: int, qseed: int, noise: float = 0.05):
    """B queries q = normalise(x_j) + noise·ε for random corpus rows j (realistic top-k margins)."""
    rng = np.random.default_rng(qseed)
    idx = rng.choice(n_rows, B, replace=False) if B <= n_rows else rng.integers(0, n_rows, B)
    x = corpus_rows(seed, idx, dim)
    x /= np.linalg.norm(x, axis=1, keepdims=True)
    eps = rng.standard_normal((B, dim)).astype(np.float32)
    eps /= np.linalg.norm(eps, axis=1, keepdims=True)
    return (x + noise * eps).astype(np.float32), idx

"""CPU oracle for the hiprag KB-search hot path -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this package, and only as the checker.  The product (youtu-rag_amd/hiprag and
libhiprag.so) never imports, links or executes anything here.

``oracle.c_*`` wrap the C restatement (hr_oracle.c, built into
oracle/_build/libhr_oracle.so by oracle/Makefile); ``oracle.ref_numpy`` is the
numpy restatement used for small cases and to cross-check the C one.  Both
follow the reference's exact store, FAISSVectorStore
(utu/rag/storage/implementations/faiss_store.py:89-199), with the canonical
summation order documented in hr_oracle.c.  Pinned against tests/golden/ (vectors
produced by the reference's own VectorRetriever, base_retriever.py:42-99).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

from . import ref_numpy  # noqa: F401

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "_build", "libhr_oracle.so")
DTYPES = {"f32": 0, "bf16": 1, "f16": 2}
METRICS = {"cosine": 0, "ip": 1, "dot": 1, "l2": 2, "euclidean": 2}
_lib = None


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        vp, i64, i32, u64 = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_uint64
        L.hro_gen_rows.argtypes = [u64, i64, i64, i32, vp]
        L.hro_normalize_rows.argtypes = [vp, i64, i32, vp]
        L.hro_quantize.argtypes = [vp, i64, i32, i32, vp]
        L.hro_build_synthetic.argtypes = [u64, i64, i64, i32, i32, i32, vp, i32]
        L.hro_search.argtypes = [vp, i32, i64, i32, vp, i32, i32, vp, i64, vp, vp, i32, i32]
        L.hro_search_synthetic.argtypes = [u64, i64, i64, i32, i32, i32, vp, i32, i32, vp, vp, i32]
        L.hro_search_synthetic.restype = i32
        L.hro_search_synthetic_masked.argtypes = [u64, i64, i64, i32, i32, i32, vp, i32, i32, vp, vp, vp, i32]
        L.hro_search_synthetic_masked.restype = i32
        L.hro_score_pairs.argtypes = [vp, i32, i32, vp, vp, vp, i64, vp, i32]
        L.hro_norm2.argtypes = [vp, i32]
        L.hro_norm2.restype = ctypes.c_double
        _lib = L
    return _lib


def _p(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


def default_threads() -> int:
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit():
        return max(1, int(env))
    return max(1, min(16, os.cpu_count() or 1))


def c_gen_rows(seed: int, row0: int, n: int, dim: int) -> np.ndarray:
    out = np.empty((n, dim), np.float32)
    lib().hro_gen_rows(seed, row0, n, dim, _p(out))
    return out


def c_normalize_rows(x: np.ndarray) -> np.ndarray:
    x = np.ascontiguousarray(x, np.float32)
    out = np.empty_like(x)
    lib().hro_normalize_rows(_p(x), x.shape[0], x.shape[1], _p(out))
    return out


def c_quantize(x: np.ndarray, dtype: str) -> np.ndarray:
    x = np.ascontiguousarray(x, np.float32)
    out = np.empty(x.shape, np.float32 if dtype == "f32" else np.uint16)
    lib().hro_quantize(_p(x), x.shape[0], x.shape[1], DTYPES[dtype], _p(out))
    return out


def c_build_synthetic(seed: int, row0: int, n: int, dim: int, dtype: str, metric: str,
                      nthreads: int | None = None) -> np.ndarray:
    out = np.empty((n, dim), np.float32 if dtype == "f32" else np.uint16)
    lib().hro_build_synthetic(seed, row0, n, dim, DTYPES[dtype], METRICS[metric], _p(out),
                              nthreads or default_threads())
    return out


def c_search(stored: np.ndarray, dtype: str, q: np.ndarray, k: int, mask: np.ndarray | None = None,
             row_offset: int = 0, nthreads: int | None = None, metric: str = "cosine"):
    """Exact top-k over stored rows; q must already be processed (normalised for cosine).
    cosine / ip score = inner product; l2 (euclidean) score = 1 - squared distance."""
    stored = np.ascontiguousarray(stored)
    q = np.ascontiguousarray(q, np.float32)
    B, dim = q.shape
    s = np.empty((B, k), np.float64)
    r = np.empty((B, k), np.int64)
    m = None if mask is None else np.ascontiguousarray(mask, np.uint64)
    lib().hro_search(_p(stored), DTYPES[dtype], stored.shape[0], dim, _p(q), B, k,
                     None if m is None else _p(m), row_offset, _p(s), _p(r), nthreads or default_threads(),
                     METRICS[metric])
    return s, r


def c_search_synthetic(seed: int, row0: int, n: int, dim: int, dtype: str, metric: str, q: np.ndarray, k: int,
                       nthreads: int | None = None, mask: np.ndarray | None = None):
    """Exact top-k over the synthetic rows [row0, row0 + n), generated on the fly; ``mask`` (optional
    uint64 bitmap, bit r = row row0 + r) restricts the search to the allowed rows."""
    q = np.ascontiguousarray(q, np.float32)
    B = q.shape[0]
    s = np.empty((B, k), np.float64)
    r = np.empty((B, k), np.int64)
    if mask is not None:
        m = np.ascontiguousarray(mask, np.uint64)
        if len(m) * 64 < n:
            raise ValueError("mask shorter than the row range")
        rc = lib().hro_search_synthetic_masked(seed, row0, n, dim, DTYPES[dtype], METRICS[metric], _p(q), B, k, _p(m),
                                               _p(s), _p(r), nthreads or default_threads())
    else:
        rc = lib().hro_search_synthetic(seed, row0, n, dim, DTYPES[dtype], METRICS[metric], _p(q), B, k, _p(s),
                                        _p(r), nthreads or default_threads())
    if rc != 0:
        raise ValueError("dim too large for the synthetic oracle")
    return s, r


def c_score_pairs(stored: np.ndarray, dtype: str, q: np.ndarray, qidx: np.ndarray, rows: np.ndarray,
                  metric: str = "cosine") -> np.ndarray:
    stored = np.ascontiguousarray(stored)
    q = np.ascontiguousarray(q, np.float32)
    qi = np.ascontiguousarray(qidx, np.int32)
    rr = np.ascontiguousarray(rows, np.int64)
    out = np.empty(len(rr), np.float64)
    lib().hro_score_pairs(_p(stored), DTYPES[dtype], q.shape[1], _p(q), _p(qi), _p(rr), len(rr), _p(out),
                          METRICS[metric])
    return out


def mask_from_bool(allowed: np.ndarray) -> np.ndarray:
    """bool[N] -> little-endian uint64 bitmap (bit r of word r>>6)."""
    allowed = np.asarray(allowed, bool)
    n = len(allowed)
    pad = (-n) % 64
    bits = np.packbits(np.concatenate([allowed, np.zeros(pad, bool)]), bitorder="little")
    return bits.view(np.uint64).copy()

"""Pure-numpy restatement of the canonical retrieval arithmetic (small cases only).

TEST INFRASTRUCTURE ONLY -- imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py as a checker; never by the product package.

It restates the same algorithm as oracle/hr_oracle.c (which it cross-checks):
  * faiss ``normalize_L2`` + ``IndexFlatIP`` semantics of the reference's exact
    store, utu/rag/storage/implementations/faiss_store.py:102-108 (add),
    :148-154 (query + search), :179-180 (similarity = inner product);
  * Chroma's "l2" space for distance_metric="euclidean" (chroma_store.py:48-53, :135):
    similarity = 1 - squared distance, exact;
  * the canonical fp64 summation order (64 strided lanes, then the butterfly
    p[i] += p[i+off], off = 32..1) that makes GPU and CPU scores bit-identical;
  * result order (score desc, row asc).
Every step is an elementwise IEEE operation, so it is bit-exact with the C version.
"""
from __future__ import annotations

import numpy as np

MASK64 = (1 << 64) - 1


def _mix64(z: np.ndarray) -> np.ndarray:
    """splitmix64 finaliser on uint64 arrays (oracle/hr_oracle.c:hro_mix64)."""
    with np.errstate(over="ignore"):
        z = z + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def gen_rows(seed: int, row0: int, n: int, dim: int) -> np.ndarray:
    """Synthetic corpus rows (integer-valued fp32), same as hro_gen_rows."""
    rows = np.arange(row0, row0 + n, dtype=np.uint64)[:, None]
    d = np.arange(dim, dtype=np.uint64)[None, :]
    with np.errstate(over="ignore"):
        key = np.uint64((seed * 0xD1B54A32D192ED03) & MASK64) + rows * np.uint64(dim) + d
    z = _mix64(key)
    m = np.uint64(0xFFFF)
    v = ((z & m).astype(np.int64) + ((z >> np.uint64(16)) & m).astype(np.int64)
         + ((z >> np.uint64(32)) & m).astype(np.int64) + (z >> np.uint64(48)).astype(np.int64) - 131070)
    return v.astype(np.float32)


def canon_sum(prod: np.ndarray) -> np.ndarray:
    """Canonical fp64 reduction over the last axis of ``prod`` (float64)."""
    dim = prod.shape[-1]
    pad = (-dim) % 64
    if pad:
        prod = np.concatenate([prod, np.zeros(prod.shape[:-1] + (pad,), np.float64)], axis=-1)
    blocks = prod.reshape(prod.shape[:-1] + (-1, 64))
    p = np.zeros(prod.shape[:-1] + (64,), np.float64)
    for j in range(blocks.shape[-2]):
        p = p + blocks[..., j, :]
    off = 32
    while off >= 1:
        p = p[..., :off] + p[..., off:2 * off]
        off >>= 1
    return p[..., 0]


def normalize_rows(x: np.ndarray) -> np.ndarray:
    """Canonical L2 normalisation (faiss normalize_L2 semantics, zero rows unchanged)."""
    x = np.asarray(x, np.float32)
    xd = x.astype(np.float64)
    n2 = canon_sum(xd * xd)
    out = x.copy()
    nz = n2 > 0
    inv = 1.0 / np.sqrt(n2[nz])
    out[nz] = (xd[nz] * inv[:, None]).astype(np.float32)
    return out


def f32_to_bf16(x: np.ndarray) -> np.ndarray:
    u = np.ascontiguousarray(x, np.float32).view(np.uint32).astype(np.uint64)
    nan = ((u & 0x7F800000) == 0x7F800000) & ((u & 0x007FFFFF) != 0)
    r = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16) & 0xFFFF
    r = np.where(nan, (u >> 16) | 0x40, r)
    return r.astype(np.uint16)


def bf16_to_f32(h: np.ndarray) -> np.ndarray:
    return (np.asarray(h, np.uint16).astype(np.uint32) << 16).view(np.float32)


def f32_to_f16(x: np.ndarray) -> np.ndarray:
    # IEEE RNE conversion; numpy's astype(float16) rounds to nearest even.
    return np.asarray(x, np.float32).astype(np.float16).view(np.uint16)


def f16_to_f32(h: np.ndarray) -> np.ndarray:
    return np.asarray(h, np.uint16).view(np.float16).astype(np.float32)


def quantize(x: np.ndarray, dtype: str) -> np.ndarray:
    if dtype == "f32":
        return np.asarray(x, np.float32).copy()
    if dtype == "bf16":
        return f32_to_bf16(x)
    if dtype == "f16":
        return f32_to_f16(x)
    raise ValueError(dtype)


def dequantize(stored: np.ndarray, dtype: str) -> np.ndarray:
    if dtype == "f32":
        return np.asarray(stored, np.float32)
    if dtype == "bf16":
        return bf16_to_f32(stored)
    return f16_to_f32(stored)


def process_rows(x: np.ndarray, metric: str, dtype: str) -> np.ndarray:
    """Rows as the store keeps them: (cosine) normalised, then quantised."""
    x = np.asarray(x, np.float32)
    if metric == "cosine":
        x = normalize_rows(x)
    return quantize(x, dtype)


def process_queries(q: np.ndarray, metric: str) -> np.ndarray:
    q = np.asarray(q, np.float32)
    return normalize_rows(q) if metric == "cosine" else q.copy()


def exact_scores(stored: np.ndarray, dtype: str, q: np.ndarray, metric: str = "cosine") -> np.ndarray:
    """B×N canonical fp64 scores of processed queries against stored rows: the inner product
    (cosine, ip), or for l2 / euclidean Chroma's similarity 1 - squared distance, evaluated as
    1 - ((|q|^2 - 2 q.x) + |x|^2) with canonical terms (chroma_store.py:48-53, :135)."""
    x = dequantize(stored, dtype).astype(np.float64)
    qd = np.asarray(q, np.float32).astype(np.float64)
    dot = canon_sum(qd[:, None, :] * x[None, :, :])
    if metric not in ("l2", "euclidean"):
        return dot
    qn2 = canon_sum(qd * qd)
    xn2 = canon_sum(x * x)
    return 1.0 - ((qn2[:, None] - 2.0 * dot) + xn2[None, :])


def search(stored: np.ndarray, dtype: str, q: np.ndarray, k: int, allowed: np.ndarray | None = None,
           row_offset: int = 0, metric: str = "cosine"):
    """Exact top-k: (scores f64 B×k, rows i64 B×k), order (score desc, row asc), -inf/-1 padding."""
    s = exact_scores(stored, dtype, q, metric)
    n = s.shape[1]
    rows = np.arange(n, dtype=np.int64)
    B = s.shape[0]
    out_s = np.full((B, k), -np.inf)
    out_r = np.full((B, k), -1, np.int64)
    for b in range(B):
        sel = rows if allowed is None else rows[allowed]
        sb = s[b, sel]
        order = np.lexsort((sel, -sb))[:k]
        out_s[b, :len(order)] = sb[order]
        out_r[b, :len(order)] = sel[order] + row_offset
    return out_s, out_r


def ivf_search(stored: np.ndarray, dtype: str, q: np.ndarray, centroids: np.ndarray, row_list: np.ndarray,
               nprobe: int, k: int, ids: np.ndarray | None = None):
    """IVF-flat restatement (FAISS IndexIVFFlat's published algorithm, faiss-cpu 1.12.0 per uv.lock:
    coarse quantizer -> the nprobe best lists -> scan those lists -> keep the k best), with the
    canonical arithmetic: coarse score = canonical fp64 q.c over the fp32 centroids, lists ordered
    (score desc, list asc); rows of the probed lists scored canonically, ordered (score desc, id asc).
    q: processed queries (B, dim); stored: processed rows (N, dim) in id order; row_list: list of
    every row.  Returns (scores f64 (B, k), ids i64 (B, k), probes i64 (B, nprobe))."""
    qd = np.asarray(q, np.float32).astype(np.float64)
    c = np.asarray(centroids, np.float32).astype(np.float64)
    coarse = canon_sum(qd[:, None, :] * c[None, :, :])
    x = dequantize(stored, dtype).astype(np.float64)
    ids = np.arange(len(stored), dtype=np.int64) if ids is None else np.asarray(ids, np.int64)
    B = qd.shape[0]
    out_s = np.full((B, k), -np.inf)
    out_r = np.full((B, k), -1, np.int64)
    probes = np.zeros((B, nprobe), np.int64)
    lists = np.arange(c.shape[0])
    for b in range(B):
        probes[b] = lists[np.lexsort((lists, -coarse[b]))][:nprobe]
        vis = np.nonzero(np.isin(row_list, probes[b]))[0]
        if len(vis) == 0:
            continue
        s = canon_sum(qd[b][None, :] * x[vis])
        order = np.lexsort((ids[vis], -s))[:k]
        out_s[b, :len(order)] = s[order]
        out_r[b, :len(order)] = ids[vis][order]
    return out_s, out_r, probes

"""Metadata where-clause -> row bitmask compiler (host side of kernel row K6).

Accepts the filter shapes the reference's callers produce:
  * plain ``{"key": value}`` (FAISS post-filter, faiss_store.py:169-176; the
    retriever's ``filters=`` kwarg, base_retriever.py:54-63), read as ``$eq``;
  * Chroma where-clauses (chroma_store.py:104-116; built by
    KBSearchToolkit._build_metadata_filters, kb_search_toolkit.py:63-96):
    ``$eq $ne $gt $gte $lt $lte $in $nin`` on fields, ``$and`` / ``$or`` lists.
A row whose metadata lacks the field matches no operator (Chroma semantics).
The result is a little-endian uint64 bitmap (bit r of word r>>6) that the scan
kernel ANDs with the tombstone bitmap, so filtered top-k is exact among the
matching rows (Chroma pre-filter semantics, not FAISS's top_k*10 post-filter).
"""
from __future__ import annotations

import numbers
from typing import Any

import numpy as np

_CMP = {"$gt": np.greater, "$gte": np.greater_equal, "$lt": np.less, "$lte": np.less_equal}


class MetadataColumns:
    """Append-only columnar cache of row metadata (rows are never re-numbered)."""

    def __init__(self):
        self.n = 0
        self._cols: dict[str, list] = {}
        self._arrays: dict[str, tuple[int, np.ndarray]] = {}

    def append(self, metas: list[dict[str, Any]]):
        for m in metas:
            for k in m:
                if k not in self._cols:
                    self._cols[k] = [None] * self.n
            for k, col in self._cols.items():
                col.append(m.get(k))
            self.n += 1

    def column(self, key: str) -> np.ndarray:
        col = self._cols.get(key)
        if col is None:
            return np.full(self.n, None, dtype=object)
        cached = self._arrays.get(key)
        if cached is not None and cached[0] == self.n:
            return cached[1]
        arr = np.empty(self.n, dtype=object)
        arr[:] = col
        self._arrays[key] = (self.n, arr)
        return arr

    def clear(self):
        self.__init__()


def _is_num(v) -> bool:
    return isinstance(v, numbers.Number) and not isinstance(v, bool)


def _eq(a, b) -> bool:
    if isinstance(a, bool) or isinstance(b, bool):  # True must not match 1
        return isinstance(a, bool) and isinstance(b, bool) and a == b
    return a == b


def _field_op(col: np.ndarray, op: str, val) -> np.ndarray:
    present = np.array([v is not None for v in col], dtype=bool)
    if op == "$eq":
        return present & np.array([_eq(v, val) for v in col], dtype=bool)
    if op == "$ne":
        return present & ~_field_op(col, "$eq", val)
    if op in ("$in", "$nin"):
        if not isinstance(val, (list, tuple, set)):
            raise ValueError(f"{op} expects a list, got {val!r}")
        vals = list(val)
        hit = np.array([any(_eq(v, x) for x in vals) for v in col], dtype=bool)
        return present & (hit if op == "$in" else ~hit)
    if op in _CMP:
        if not _is_num(val):
            raise ValueError(f"{op} expects a number, got {val!r}")
        num = np.array([_is_num(v) for v in col], dtype=bool)
        out = np.zeros(len(col), dtype=bool)
        if num.any():
            out[num] = _CMP[op](col[num].astype(np.float64), float(val))
        return out
    raise ValueError(f"unsupported where operator {op!r}")


def evaluate(where: dict[str, Any], cols: MetadataColumns) -> np.ndarray:
    """bool[n]: rows matching ``where``."""
    if not isinstance(where, dict):
        raise ValueError(f"where clause must be a dict, got {type(where).__name__}")
    out = np.ones(cols.n, dtype=bool)
    for key, cond in where.items():
        if key in ("$and", "$or"):
            if not isinstance(cond, list) or not cond:
                raise ValueError(f"{key} expects a non-empty list")
            parts = [evaluate(c, cols) for c in cond]
            m = np.logical_and.reduce(parts) if key == "$and" else np.logical_or.reduce(parts)
        elif key.startswith("$"):
            raise ValueError(f"unsupported top-level operator {key!r}")
        else:
            col = cols.column(key)
            if isinstance(cond, dict) and cond and all(k.startswith("$") for k in cond):
                m = np.ones(cols.n, dtype=bool)
                for op, val in cond.items():
                    m &= _field_op(col, op, val)
            else:
                m = _field_op(col, "$eq", cond)
        out &= m
    return out


def to_bitmap(mask: np.ndarray) -> np.ndarray:
    """bool[n] -> uint64 bitmap, bit r of word r>>6."""
    mask = np.asarray(mask, dtype=bool)
    pad = (-len(mask)) % 64
    return np.packbits(np.concatenate([mask, np.zeros(pad, bool)]), bitorder="little").view(np.uint64).copy()

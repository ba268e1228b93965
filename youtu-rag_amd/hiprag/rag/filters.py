"""Metadata where-clause -> row bitmap compiler (host side of kernel row K6).

Accepts the filter shapes the reference's callers produce:
  * plain ``{"key": value}`` (FAISS post-filter, faiss_store.py:169-176; the
    retriever's ``filters=`` kwarg, base_retriever.py:54-63), read as ``$eq``;
  * Chroma where-clauses (chroma_store.py:104-116; built by
    KBSearchToolkit._build_metadata_filters, kb_search_toolkit.py:63-96):
    ``$eq $ne $gt $gte $lt $lte $in $nin`` on fields, ``$and`` / ``$or`` lists.
A row whose metadata lacks the field matches no operator (Chroma semantics); ``True`` does
not match ``1``; the order comparisons apply to numbers (not bools) only.

Layout: a columnar, append-only cache.  Every key is a column of int32 *codes* (one per
distinct value, -1 = absent) plus a float64 column of numeric values (NaN = not a number),
so a predicate is one vectorised compare, never a per-row Python call.  Rows are never
re-numbered and their metadata never changes, so the packed bitmap of every leaf predicate
(key, op, value) is cached and, when rows are appended, extended over the new rows only: a
repeated filter -- ``kb_file_search``'s ``index_type == "index_summary"``, a ``source`` or
``document_id`` -- costs a few word-wise ANDs of cached bitmaps (0.16 MB per million rows).
The result is a little-endian uint64 bitmap (bit r of word r>>6) that the scan kernel ANDs
with the tombstone bits, so a filtered top-k is exact among the matching rows (Chroma
pre-filter semantics, not FAISS's top_k*10 post-filter).
"""
from __future__ import annotations

import json
import numbers
from collections import OrderedDict
from typing import Any

import numpy as np

_CMP = {"$gt": np.greater, "$gte": np.greater_equal, "$lt": np.less, "$lte": np.less_equal}
_ALL = np.uint64(0xFFFFFFFFFFFFFFFF)


def _is_num(v) -> bool:
    return isinstance(v, numbers.Number) and not isinstance(v, bool)


def _vkey(v):
    """Dictionary key of a metadata value with Python equality, except that bools only equal bools
    (1 == 1.0 share a key; True and 1 do not)."""
    if isinstance(v, bool):
        return ("b", v)
    if _is_num(v):
        return ("n", v)
    if isinstance(v, str):
        return ("s", v)
    try:
        hash(v)
        return ("o", v)
    except TypeError:
        return ("j", json.dumps(v, sort_keys=True, default=str))


class _Column:
    __slots__ = ("codes", "num", "dict")

    def __init__(self, cap: int):
        self.codes = np.full(cap, -1, np.int32)
        self.num = np.full(cap, np.nan, np.float64)
        self.dict: dict = {}

    def grow(self, cap: int):
        if cap > len(self.codes):
            c = np.full(cap, -1, np.int32)
            c[: len(self.codes)] = self.codes
            x = np.full(cap, np.nan, np.float64)
            x[: len(self.num)] = self.num
            self.codes, self.num = c, x


def n_words(n: int) -> int:
    return (n + 63) // 64


def pack(mask: np.ndarray) -> np.ndarray:
    """bool[n] -> uint64 words, bit r of word r>>6 (tail bits zero)."""
    mask = np.asarray(mask, dtype=bool)
    pad = (-len(mask)) % 64
    if pad:
        mask = np.concatenate([mask, np.zeros(pad, bool)])
    return np.packbits(mask, bitorder="little").view(np.uint64).copy()


def unpack(words: np.ndarray, n: int) -> np.ndarray:
    return np.unpackbits(np.asarray(words, np.uint64).view(np.uint8), bitorder="little")[:n].astype(bool)


def _tail_fix(words: np.ndarray, n: int) -> np.ndarray:
    if n % 64 and len(words):
        words[-1] &= np.uint64((1 << (n % 64)) - 1)
    return words


class MetadataColumns:
    """Append-only columnar cache of row metadata (rows are never re-numbered)."""

    CACHE_ENTRIES = 256

    def __init__(self):
        self.n = 0
        self._cap = 0
        self._cols: dict[str, _Column] = {}
        self._cache: OrderedDict = OrderedDict()  # leaf predicate -> [rows covered, words]

    def append(self, metas: list[dict[str, Any]]):
        n0, m = self.n, len(metas)
        if n0 + m > self._cap:
            self._cap = max(n0 + m, 2 * self._cap, 1024)
            for c in self._cols.values():
                c.grow(self._cap)
        cols = self._cols
        for i, meta in enumerate(metas):
            r = n0 + i
            for k, v in meta.items():
                if v is None:
                    continue
                c = cols.get(k)
                if c is None:
                    c = cols[k] = _Column(self._cap)
                vk = _vkey(v)
                code = c.dict.get(vk)
                if code is None:
                    code = c.dict[vk] = len(c.dict)
                c.codes[r] = code
                if _is_num(v):
                    c.num[r] = float(v)
        self.n = n0 + m

    def clear(self):
        self.__init__()

    def column(self, key: str) -> np.ndarray:
        """Values of one key as an object array (None = absent) -- diagnostics and tests."""
        c = self._cols.get(key)
        out = np.full(self.n, None, dtype=object)
        if c is None:
            return out
        inv = [None] * len(c.dict)
        for vk, code in c.dict.items():
            inv[code] = vk[1] if vk[0] != "j" else json.loads(vk[1])
        codes = c.codes[: self.n]
        for r in np.nonzero(codes >= 0)[0]:
            out[r] = inv[codes[r]]
        return out

    # -- leaf predicates (cached bitmaps)
    def _leaf_bool(self, key: str, op: str, arg, r0: int, r1: int) -> np.ndarray:
        c = self._cols.get(key)
        if c is None:
            return np.zeros(r1 - r0, bool)
        codes = c.codes[r0:r1]
        if op == "present":
            return codes >= 0
        if op == "in":  # arg: frozenset of codes
            if not arg:
                return np.zeros(r1 - r0, bool)
            if len(arg) <= 8:  # a few values ($in of some files): OR of compares beats np.isin's sort
                it = iter(arg)
                out = codes == next(it)
                for c in it:
                    out |= codes == c
                return out
            return np.isin(codes, np.fromiter(arg, np.int32, len(arg)))
        with np.errstate(invalid="ignore"):
            return _CMP[op](c.num[r0:r1], arg)  # NaN (absent / not a number) compares False

    def leaf(self, key: str, op: str, arg) -> np.ndarray:
        """Packed bitmap of one field predicate over all n rows, cached and extended on append."""
        ck = (key, op, arg)
        ent = self._cache.get(ck)
        n, nw = self.n, n_words(self.n)
        if ent is not None and ent[0] == n:
            self._cache.move_to_end(ck)
            return ent[1]
        if ent is None:
            w0, words = 0, np.zeros(nw, np.uint64)
        else:
            w0 = ent[0] // 64  # re-evaluate from the word holding the first new row
            words = np.zeros(nw, np.uint64)
            words[: len(ent[1])] = ent[1]
        if n > w0 * 64:
            words[w0:] = pack(self._leaf_bool(key, op, arg, w0 * 64, n))
        self._cache[ck] = [n, words]
        self._cache.move_to_end(ck)
        while len(self._cache) > self.CACHE_ENTRIES:
            self._cache.popitem(last=False)
        return words

    def codes_of(self, key: str, vals) -> frozenset:
        c = self._cols.get(key)
        if c is None:
            return frozenset()
        out = set()
        for v in vals:
            code = c.dict.get(_vkey(v))
            if code is not None:
                out.add(code)
        return frozenset(out)

    def all_words(self) -> np.ndarray:
        return _tail_fix(np.full(n_words(self.n), _ALL, np.uint64), self.n)


def _field_op(cols: MetadataColumns, key: str, op: str, val) -> np.ndarray:
    if op == "$eq":
        return cols.leaf(key, "in", cols.codes_of(key, [val]))
    if op == "$ne":
        return cols.leaf(key, "present", None) & ~cols.leaf(key, "in", cols.codes_of(key, [val]))
    if op in ("$in", "$nin"):
        if not isinstance(val, (list, tuple, set)):
            raise ValueError(f"{op} expects a list, got {val!r}")
        hit = cols.leaf(key, "in", cols.codes_of(key, val))
        return hit if op == "$in" else cols.leaf(key, "present", None) & ~hit
    if op in _CMP:
        if not _is_num(val):
            raise ValueError(f"{op} expects a number, got {val!r}")
        return cols.leaf(key, op, float(val))
    raise ValueError(f"unsupported where operator {op!r}")


def evaluate_words(where: dict[str, Any], cols: MetadataColumns) -> np.ndarray:
    """uint64 words (bit r = row r matches ``where``), tail bits zero."""
    if not isinstance(where, dict):
        raise ValueError(f"where clause must be a dict, got {type(where).__name__}")
    out = None
    for key, cond in where.items():
        if key in ("$and", "$or"):
            if not isinstance(cond, list) or not cond:
                raise ValueError(f"{key} expects a non-empty list")
            parts = [evaluate_words(c, cols) for c in cond]
            m = parts[0].copy()
            for p in parts[1:]:
                if key == "$and":
                    m &= p
                else:
                    m |= p
        elif key.startswith("$"):
            raise ValueError(f"unsupported top-level operator {key!r}")
        elif isinstance(cond, dict) and cond and all(k.startswith("$") for k in cond):
            m = None
            for op, val in cond.items():
                w = _field_op(cols, key, op, val)
                m = w.copy() if m is None else (m & w)
        else:
            m = _field_op(cols, key, "$eq", cond)
        out = m.copy() if out is None else (out & m)
    if out is None:
        out = cols.all_words()
    return _tail_fix(out, cols.n)


def evaluate(where: dict[str, Any], cols: MetadataColumns) -> np.ndarray:
    """bool[n]: rows matching ``where``."""
    return unpack(evaluate_words(where, cols), cols.n)


def to_bitmap(mask: np.ndarray) -> np.ndarray:
    """bool[n] -> uint64 bitmap, bit r of word r>>6."""
    return pack(mask)

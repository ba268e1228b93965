"""On-disk format of a HipVectorStore collection: generation snapshots + an append-only journal.

Replaces the persistence of the reference's stores -- Chroma's PersistentClient directory
(chroma.sqlite3 WAL + HNSW segments, chroma_store.py:41-44, :298-306) and FAISS's
``write_index`` + pickle (faiss_store.py:61-87, rewritten in full on every save) -- with:

  <collection>.manifest.json      {"gen": g, "n_rows": n, dim, dtype, metric}; replaced
                                  atomically (tmp + fsync + rename) LAST, so it always names
                                  a complete snapshot
  <collection>.g<g>.hri           the device index of generation g (hr_index_save: tiled rows
                                  + live bits, itself written tmp + fsync + rename)
  <collection>.g<g>.rows.jsonl    header {"gen", "n_rows", ...} + one record per row (null =
                                  deleted)
  <collection>.g<g>.emb.npy       optional raw fp32 embeddings (keep_embeddings)
  <collection>.g<g>.journal       adds and deletes since the snapshot, append-only

``add_chunks`` appends its records and fp32 vectors to the journal and ``delete*`` appends the
deleted rows: O(chunk) bytes per call instead of a rewrite of the whole index (the reference's
ingest calls delete + add once per document, processors.py:364, :418).  The journal is folded
into a new generation when it outgrows a fraction of the snapshot (or on ``flush``/bulk ingest
end).  Every journal entry carries its length and a CRC32; a torn tail (a crash mid-append) is
dropped on load.  Loading checks that the index, the row table and the manifest agree on the row
count and takes dim / dtype / metric from the files, not from the caller's config.
"""
from __future__ import annotations

import io
import json
import os
import re
import struct
import zlib

import numpy as np

MAGIC = b"HRJ1"
_HDR = struct.Struct("<4sBxxxQI")  # magic, type, payload length, crc32
ADD, DEL = 1, 2
FORMAT = "hiprag-store-2"


def fsync_write(path: str, data: bytes | None = None, writer=None) -> None:
    """Write ``path`` crash-safely: <path>.tmp, fsync, rename."""
    tmp = path + ".tmp"
    with open(tmp, "wb") as f:
        if writer is not None:
            writer(f)
        else:
            f.write(data)
        f.flush()
        os.fsync(f.fileno())
    os.replace(tmp, path)
    _fsync_dir(os.path.dirname(path) or ".")


def _fsync_dir(d: str) -> None:
    try:
        fd = os.open(d, os.O_RDONLY)
    except OSError:
        return
    try:
        os.fsync(fd)
    except OSError:
        pass
    finally:
        os.close(fd)


class Paths:
    def __init__(self, directory: str, collection: str):
        self.dir = directory
        self.base = os.path.join(directory, collection)

    @property
    def manifest(self):
        return self.base + ".manifest.json"

    def gen(self, g: int, ext: str) -> str:
        return f"{self.base}.g{g}.{ext}"

    # round-1 layout (one .hri + one .rows.jsonl, rewritten on every save)
    @property
    def legacy(self):
        return self.base + ".hri", self.base + ".rows.jsonl"

    def all_files(self) -> list[str]:
        d = self.dir
        if not os.path.isdir(d):
            return []
        # exactly this collection's names: a prefix match would also take a sibling collection's files
        # ("docs" vs "docs.gov")
        pat = re.compile(re.escape(os.path.basename(self.base))
                         + r"\.(manifest\.json|g\d+\.(hri|rows\.jsonl|emb\.npy|journal)|hri|rows\.jsonl)(\.tmp)?")
        return [os.path.join(d, f) for f in os.listdir(d) if pat.fullmatch(f)]


class Journal:
    """Append-only log of the adds and deletes since the last snapshot."""

    def __init__(self, path: str, fsync: bool = True):
        self.path, self.fsync = path, fsync
        self._f = None

    @property
    def size(self) -> int:
        return self._f.tell() if self._f is not None else (os.path.getsize(self.path) if os.path.exists(self.path) else 0)

    def _append(self, typ: int, payload: bytes) -> int:
        if self._f is None:
            self._f = open(self.path, "ab")
        self._f.write(_HDR.pack(MAGIC, typ, len(payload), zlib.crc32(payload)) + payload)
        self._f.flush()
        if self.fsync:
            os.fsync(self._f.fileno())
        return _HDR.size + len(payload)

    def append_add(self, records: list[dict], vectors: np.ndarray) -> int:
        v = np.ascontiguousarray(vectors, np.float32)
        js = json.dumps(records).encode()
        payload = struct.pack("<Q", len(js)) + js + struct.pack("<QQ", *v.shape) + v.tobytes()
        return self._append(ADD, payload)

    def append_delete(self, rows) -> int:
        return self._append(DEL, np.ascontiguousarray(np.asarray(rows, np.int64)).tobytes())

    def close(self):
        if self._f is not None:
            self._f.close()
            self._f = None

    @staticmethod
    def replay(path: str):
        """Yield ("add", records, vectors) / ("del", rows) in order; a torn or corrupt tail is cut off
        (the file is truncated to the last complete entry)."""
        if not os.path.exists(path):
            return
        good = 0
        with open(path, "rb") as f:
            data = f.read()
        pos = 0
        while pos + _HDR.size <= len(data):
            magic, typ, ln, crc = _HDR.unpack_from(data, pos)
            end = pos + _HDR.size + ln
            if magic != MAGIC or end > len(data):
                break
            payload = data[pos + _HDR.size:end]
            if zlib.crc32(payload) != crc:
                break
            if typ == ADD:
                (jl,) = struct.unpack_from("<Q", payload, 0)
                records = json.loads(payload[8:8 + jl].decode())
                n, dim = struct.unpack_from("<QQ", payload, 8 + jl)
                vec = np.frombuffer(payload, np.float32, count=n * dim, offset=8 + jl + 16).reshape(n, dim)
                yield "add", records, vec
            elif typ == DEL:
                yield "del", np.frombuffer(payload, np.int64), None
            else:
                break
            pos = good = end
        if good < len(data):
            with open(path, "r+b") as f:
                f.truncate(good)


def write_rows(path: str, header: dict, records: list) -> None:
    def w(f):
        buf = io.TextIOWrapper(f, encoding="utf-8", write_through=True)
        buf.write(json.dumps(header) + "\n")
        for rec in records:
            buf.write(json.dumps(rec) + "\n")
        buf.flush()
        buf.detach()

    fsync_write(path, writer=w)


def read_rows(path: str) -> tuple[dict, list]:
    with open(path, encoding="utf-8") as f:
        header = json.loads(f.readline())
        records = [json.loads(line) for line in f]
    return header, records

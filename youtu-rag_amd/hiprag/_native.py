"""ctypes bindings to libhiprag.so (the HIP/gfx950 vector index).

Declarations: include/hiprag.h.  ctypes releases the GIL for the duration of
every foreign call, so a blocking search does not stall other Python threads.
There is no CPU fallback: if the shared library or a GPU is missing, the
constructors raise.
"""
from __future__ import annotations

import ctypes
import os
import threading

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libhiprag.so")

DTYPES = {"f32": 0, "float32": 0, "fp32": 0, "bf16": 1, "bfloat16": 1, "f16": 2, "float16": 2, "fp16": 2}
METRICS = {"cosine": 0, "ip": 1, "dot": 1, "euclidean": 2, "l2": 2}
HR_MAX_K = 128   # include/hiprag.h
HR_MAX_KC = 256


def kc_for_k(k: int, dim: int = 0) -> int:
    """Per-shard candidate count for top-k (hr_kc_for_k_dim): k + max(16, k // 2) rounded up to 32 (32
    for k <= 16), the margin max(20, k) from 2048 dims on, at most HR_MAX_KC (tests/test_native_abi.py
    checks it against the library)."""
    wide = 2 if (dim + 63) // 64 * 64 >= 2048 else 1
    return min(HR_MAX_KC, (k + max(20 if wide == 2 else 16, wide * k // 2) + 31) // 32 * 32)


CAND_DTYPE = np.dtype([("score", "<f8"), ("row", "<i8")])  # matches hr::Cand

E_INVALID, E_HIP, E_UNSUPPORTED, E_OVERFLOW, E_IO, E_BUSY = -1, -2, -3, -4, -5, -6

# every symbol include/hiprag.h declares (checked by tests/test_native_abi.py)
EXPORTS = [
    "hr_index_create", "hr_index_reserve", "hr_index_add", "hr_index_add_synthetic", "hr_index_add_device",
    "hr_index_remove", "hr_index_search", "hr_index_search_device", "hr_index_size", "hr_index_get_rows",
    "hr_index_save", "hr_index_load", "hr_index_destroy", "hr_index_search_shard", "hr_index_search_shard_collect",
    "hr_merge_candidates", "hr_pool_normalize", "hr_pool_normalize_packed", "hr_hash_words", "hr_index_set_scan_timing", "hr_index_take_scan_times", "hr_index_last_scan_ms",
    "hr_device_count", "hr_index_debug_approx", "hr_index_last_candidates", "hr_last_error", "hr_abi_version",
    "hr_kc_for_k", "hr_merge_candidates_strided", "hr_index_search_shard_async", "hr_index_add_device_at",
    "hr_gen_rows_device", "hr_ivf_search", "hr_topk_records", "hr_index_search_shard_async_ev", "hr_index_stats",
    "hr_add_layernorm", "hr_index_info", "hr_index_graph_replays", "hr_index_wide_launches", "hr_kc_for_k_dim",
    "hr_index_search_submit", "hr_index_search_finalize", "hr_index_host_us", "hr_index_search_submit_host",
    "hr_index_search_collect", "hr_index_search_poll", "hr_index_set_persist", "hr_index_persist_close",
    "hr_index_persist_stats", "hr_index_persist_trace", "hr_index_wave_tiles", "hr_index_set_cu_mask",
    "hr_stream_create_cu_mask", "hr_stream_destroy", "hr_index_set_q256", "hr_index_q256_launches",
    "hr_index_search_shard_exact", "hr_merge_sorted", "hr_memcpy_async", "hr_attn_varlen", "hr_gelu_erf",
]

_lib = None
_lib_lock = threading.Lock()


def cu_mask_words(cus) -> np.ndarray:
    """uint32 mask words of a CU list (bit i of word j = CU 32 j + i)."""
    cus = [int(c) for c in cus]
    words = np.zeros(max(cus) // 32 + 1, np.uint32)
    for c in cus:
        words[c // 32] |= np.uint32(1 << (c % 32))
    return words


def create_cu_stream(device: int, cus) -> int:
    """A raw HIP stream of `device` restricted to the CUs in `cus` (wrap it with torch.cuda.ExternalStream); release
    it with destroy_stream."""
    lib = load_library()
    words = cu_mask_words(cus)
    out = ctypes.c_void_p()
    _check(lib.hr_stream_create_cu_mask(int(device), words.ctypes.data, len(words), ctypes.byref(out)))
    return int(out.value)


def destroy_stream(stream: int) -> None:
    """Wait for the stream's work and destroy it (hr_stream_destroy).  Free first every pinned host tensor that a
    non_blocking torch copy ran on this stream for: torch's pinned-memory allocator records those streams and uses
    them again when the tensor is freed (a destroyed stream there crashed the interpreter at exit)."""
    _check(load_library().hr_stream_destroy(ctypes.c_void_p(stream)))


def memcpy_async(dst_ptr: int, src_ptr: int, nbytes: int, stream: int = 0) -> None:
    """Asynchronous copy on `stream` (hr_memcpy_async), outside torch's allocators' stream bookkeeping."""
    _check(load_library().hr_memcpy_async(ctypes.c_void_p(dst_ptr), ctypes.c_void_p(src_ptr), int(nbytes),
                                          ctypes.c_void_p(stream or None)))


class NativeError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"hiprag error {code}: {msg}")
        self.code = code


class BusyError(NativeError):
    """hr_index_search_submit_host found the handle held by another call (it never waits)."""


def load_library(path: str | None = None):
    """Load libhiprag.so (raises OSError if it was not built: run __graft_entry__.build())."""
    global _lib
    with _lib_lock:
        if _lib is not None:
            return _lib
        # One HIP runtime per process: torch bundles its own libamdhip64.so.7 (same SONAME as
        # /opt/rocm's).  Loading torch first makes libhiprag.so bind to that same runtime, so
        # torch tensors, streams and RCCL interoperate with our kernels.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        p = path or os.environ.get("HIPRAG_LIB_OVERRIDE") or LIB_PATH  # override: A/B timing builds only
        if not os.path.exists(p):
            raise OSError(f"{p} not found; build it with `make -C youtu-rag_amd/csrc` or __graft_entry__.build()")
        L = ctypes.CDLL(p)
        vp, i32, i64, u64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_uint64
        pp = ctypes.POINTER(ctypes.c_void_p)
        sig = {
            "hr_index_create": [i32, i32, i32, i32, vp, pp],
            "hr_index_reserve": [vp, i64],
            "hr_index_add": [vp, vp, i64, vp],
            "hr_index_add_synthetic": [vp, u64, i64, i64, vp],
            "hr_index_add_device": [vp, vp, i64, vp, vp],
            "hr_index_remove": [vp, vp, i64],
            "hr_index_search": [vp, vp, i32, i32, vp, vp, vp],
            "hr_index_search_device": [vp, vp, i32, i32, vp, vp, vp, vp],
            "hr_index_search_submit": [vp, vp, i32, i32, vp, vp, vp, vp],
            "hr_index_search_finalize": [vp, i64],
            "hr_index_host_us": [vp, vp],
            "hr_index_search_submit_host": [vp, vp, i32, i32, i32, vp],
            "hr_index_search_collect": [vp, i64, vp, vp],
            "hr_index_search_poll": [vp, i64, vp],
            "hr_index_set_persist": [vp, i32],
            "hr_index_persist_close": [vp],
            "hr_index_persist_stats": [vp, vp],
            "hr_index_persist_trace": [vp, ctypes.c_int, vp, vp],
            "hr_index_wave_tiles": [vp, vp, i32, vp],
            "hr_index_set_cu_mask": [vp, vp, i32],
            "hr_stream_create_cu_mask": [i32, vp, i32, pp],
            "hr_stream_destroy": [vp],
            "hr_memcpy_async": [vp, vp, i64, vp],
            "hr_attn_varlen": [vp, i32, vp, i32, i32, i32, i32, ctypes.c_float, vp, vp],
            "hr_gelu_erf": [vp, i32, i64, vp],
            "hr_index_set_q256": [vp, i32],
            "hr_index_q256_launches": [vp, vp],
            "hr_index_size": [vp, vp, vp],
            "hr_index_info": [vp, vp, vp, vp, vp],
            "hr_index_get_rows": [vp, vp, i64, vp],
            "hr_index_save": [vp, ctypes.c_char_p],
            "hr_index_load": [ctypes.c_char_p, i32, vp, pp],
            "hr_index_search_shard": [vp, vp, i32, i32, i32, vp, i64, vp, vp, vp],
            "hr_index_search_shard_async": [vp, vp, i32, i32, i32, vp, i64, vp, vp, vp, vp],
            "hr_index_search_shard_async_ev": [vp, vp, i32, i32, i32, vp, i64, vp, vp, vp, vp, vp],
            "hr_index_add_device_at": [vp, vp, i64, vp, i64, vp],
            "hr_gen_rows_device": [u64, i64, i64, i32, vp, vp],
            "hr_topk_records": [vp, vp, i64, i32, i32, vp, vp],
            "hr_ivf_search": [vp, vp, i32, vp, i64, vp, vp, i32, i32, i32, vp, vp, vp, vp, vp],
            "hr_index_search_shard_collect": [vp, vp, i32, vp, i32, vp, i64, vp, vp, vp],
            "hr_index_search_shard_exact": [vp, vp, i32, i32, vp, i64, vp, vp],
            "hr_merge_sorted": [i32, vp, i64, i32, i32, i32, i32, vp, vp, vp],
            "hr_merge_candidates": [i32, vp, vp, i32, i32, i32, i32, vp, vp, vp, vp, vp],
            "hr_merge_candidates_strided": [i32, vp, vp, i64, i64, i32, i32, i32, i32, vp, vp, vp, vp, vp],
            "hr_pool_normalize": [vp, i32, vp, i32, i32, i32, i32, vp, vp],
            "hr_pool_normalize_packed": [vp, i32, vp, i32, i32, i32, vp, vp],
            "hr_hash_words": [vp, vp, i64, i64, i64, i64, i64, i64, vp, i64, vp],
            "hr_index_last_scan_ms": [vp, vp, vp],
            "hr_index_take_scan_times": [vp, vp, vp, i32, vp],
            "hr_index_set_scan_timing": [vp, i32],
            "hr_device_count": [vp],
            "hr_index_debug_approx": [vp, vp, i32, vp, vp],
            "hr_index_last_candidates": [vp, vp, vp],
            "hr_index_stats": [vp, vp],
            "hr_index_graph_replays": [vp, vp],
            "hr_index_wide_launches": [vp, vp],
            "hr_add_layernorm": [vp, vp, vp, vp, vp, i64, i32, ctypes.c_float, i32, vp],
        }
        for name, args in sig.items():
            if p != (path or LIB_PATH) and not hasattr(L, name):
                continue  # an A/B timing build of an older source (HIPRAG_LIB_OVERRIDE) may lack newer entry points
            fn = getattr(L, name)
            fn.argtypes = args
            fn.restype = i32
        L.hr_index_destroy.argtypes = [vp]
        L.hr_index_destroy.restype = None
        L.hr_last_error.argtypes = []
        L.hr_last_error.restype = ctypes.c_char_p
        L.hr_abi_version.restype = i32
        L.hr_kc_for_k.argtypes = [i32]
        L.hr_kc_for_k.restype = i32
        L.hr_kc_for_k_dim.argtypes = [i32, i32]
        L.hr_kc_for_k_dim.restype = i32
        _lib = L
        return L


def _check(rc: int):
    if rc != 0:
        msg = (load_library().hr_last_error() or b"").decode(errors="replace")
        if rc == E_INVALID:
            raise ValueError(msg)
        if rc == E_UNSUPPORTED:
            raise NotImplementedError(msg)
        if rc == E_BUSY:
            raise BusyError(rc, msg)
        raise NativeError(rc, msg)


def _ptr(a: np.ndarray | None):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def device_count() -> int:
    n = ctypes.c_int(0)
    _check(load_library().hr_device_count(ctypes.byref(n)))
    return n.value


class NativeIndex:
    """One device shard of the vector index (an hr_index handle)."""

    def __init__(self, dim: int, dtype: str = "bf16", metric: str = "cosine", device: int = 0,
                 devices: list[int] | None = None, _handle=None):
        """One index handle.  ``devices`` (GPU ids, repeats allowed) shards its rows over several
        GPUs inside the handle (hr_index_create with n_dev > 1); default: the single ``device``."""
        self.lib = load_library()
        self.devices = [int(d) for d in devices] if devices else [int(device)]
        self.dim, self.dtype, self.metric, self.device = int(dim), dtype, metric, self.devices[0]
        if _handle is not None:
            self._h = _handle
            return
        if dtype not in DTYPES:
            raise ValueError(f"unknown dtype {dtype!r}")
        if metric not in METRICS:
            raise ValueError(f"unknown metric {metric!r}")
        h = ctypes.c_void_p()
        dev = (ctypes.c_int * len(self.devices))(*self.devices)
        _check(self.lib.hr_index_create(self.dim, DTYPES[dtype], METRICS[metric], len(self.devices), dev,
                                        ctypes.byref(h)))
        self._h = h

    # -- lifecycle
    def close(self):
        if getattr(self, "_h", None):
            self.lib.hr_index_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -- data
    def reserve(self, rows: int):
        _check(self.lib.hr_index_reserve(self._h, int(rows)))

    def add(self, rows: np.ndarray) -> int:
        rows = np.ascontiguousarray(rows, np.float32)
        if rows.ndim != 2 or rows.shape[1] != self.dim:
            raise ValueError(f"rows must be (n, {self.dim}) float32")
        first = ctypes.c_int64(0)
        _check(self.lib.hr_index_add(self._h, _ptr(rows), rows.shape[0], ctypes.byref(first)))
        return first.value

    def add_device(self, rows_ptr: int, n: int, stream: int = 0) -> int:
        """Add n fp32 rows (row-major, dim wide) already in device memory; ordered after `stream`."""
        first = ctypes.c_int64(0)
        _check(self.lib.hr_index_add_device(self._h, ctypes.c_void_p(int(rows_ptr)), int(n), ctypes.byref(first),
                                            ctypes.c_void_p(int(stream))))
        return first.value

    def add_device_at(self, rows_ptr: int, n: int, dest_ptr: int, n_rows_after: int, stream: int = 0) -> None:
        """Store n fp32 device rows at the int64 device positions dest (IVF list placement)."""
        _check(self.lib.hr_index_add_device_at(self._h, ctypes.c_void_p(int(rows_ptr)), int(n),
                                               ctypes.c_void_p(int(dest_ptr)), int(n_rows_after),
                                               ctypes.c_void_p(int(stream))))

    def ivf_search(self, centroids_ptr: int, nlist: int, list_tiles_ptr: int, max_list_tiles: int, ids_ptr: int,
                   q_ptr: int, B: int, nprobe: int, k: int, cand_ptr: int, bound_ptr: int, probes_ptr: int = 0,
                   mask_ptr: int = 0, stream: int = 0) -> None:
        """IVF-flat search of the list-ordered rows of this index (hr_ivf_search)."""
        _check(self.lib.hr_ivf_search(self._h, ctypes.c_void_p(centroids_ptr), int(nlist),
                                      ctypes.c_void_p(list_tiles_ptr), int(max_list_tiles), ctypes.c_void_p(ids_ptr),
                                      ctypes.c_void_p(q_ptr), int(B), int(nprobe), int(k),
                                      ctypes.c_void_p(mask_ptr or None), ctypes.c_void_p(cand_ptr),
                                      ctypes.c_void_p(bound_ptr), ctypes.c_void_p(probes_ptr or None),
                                      ctypes.c_void_p(stream or None)))

    def add_synthetic(self, seed: int, global_row0: int, n: int) -> int:
        first = ctypes.c_int64(0)
        _check(self.lib.hr_index_add_synthetic(self._h, int(seed), int(global_row0), int(n), ctypes.byref(first)))
        return first.value

    def remove(self, rows) -> None:
        r = np.ascontiguousarray(np.asarray(rows, np.int64).reshape(-1))
        _check(self.lib.hr_index_remove(self._h, _ptr(r), len(r)))

    def size(self) -> tuple[int, int]:
        n, live = ctypes.c_int64(0), ctypes.c_int64(0)
        _check(self.lib.hr_index_size(self._h, ctypes.byref(n), ctypes.byref(live)))
        return n.value, live.value

    def get_rows(self, rows) -> np.ndarray:
        r = np.ascontiguousarray(np.asarray(rows, np.int64).reshape(-1))
        out = np.empty((len(r), self.dim), np.float32)
        _check(self.lib.hr_index_get_rows(self._h, _ptr(r), len(r), _ptr(out)))
        return out

    # -- search
    def search(self, q: np.ndarray, k: int, mask: np.ndarray | None = None) -> tuple[np.ndarray, np.ndarray]:
        q = np.ascontiguousarray(q, np.float32)
        if q.ndim == 1:
            q = q[None, :]
        if q.shape[1] != self.dim:
            raise ValueError(f"query dim {q.shape[1]} != index dim {self.dim}")
        B = q.shape[0]
        s = np.empty((B, k), np.float32)
        r = np.empty((B, k), np.int64)
        m = None
        if mask is not None:
            m = np.ascontiguousarray(mask, np.uint64).reshape(-1)
            n_rows = self.size()[0]
            if len(m) * 64 < n_rows:  # the library reads one bit per index row
                raise ValueError(f"row mask has {len(m)} words, the index {n_rows} rows "
                                 f"(needs {(n_rows + 63) // 64})")
        _check(self.lib.hr_index_search(self._h, _ptr(q), B, int(k), _ptr(m), _ptr(s), _ptr(r)))
        return s, r

    def search_device(self, q_ptr: int, B: int, k: int, scores_ptr: int, rows_ptr: int, mask_ptr: int = 0,
                      stream: int = 0) -> None:
        _check(self.lib.hr_index_search_device(self._h, ctypes.c_void_p(q_ptr), int(B), int(k),
                                               ctypes.c_void_p(mask_ptr or None), ctypes.c_void_p(scores_ptr),
                                               ctypes.c_void_p(rows_ptr), ctypes.c_void_p(stream or None)))

    def search_submit(self, q_ptr: int, B: int, k: int, scores_ptr: int, rows_ptr: int, stream: int = 0) -> int:
        """Pipelined search_device (no mask): enqueue a batch, return its ticket.  A multi-device handle
        keeps two batches in flight (one host thread per shard); the outputs are final once
        search_finalize(ticket) returns.  A single-device handle finishes the batch here (ticket 0)."""
        t = ctypes.c_int64(0)
        _check(self.lib.hr_index_search_submit(self._h, ctypes.c_void_p(q_ptr), int(B), int(k),
                                               ctypes.c_void_p(scores_ptr), ctypes.c_void_p(rows_ptr),
                                               ctypes.c_void_p(stream or None), ctypes.byref(t)))
        return t.value

    def search_submit_host(self, q: np.ndarray, k: int, notify_fd: int = -1) -> int:
        """Asynchronous search of host queries (single-device handle, no mask): returns a ticket at once;
        when the batch's results reach host memory an 8-byte 1 is written to notify_fd (an eventfd).
        At most two batches in flight, collected in any order (a third raises BusyError).  Raises
        NotImplementedError where hr_index_search must serve (empty index, multi-device handle)."""
        q = np.ascontiguousarray(q, np.float32)
        if q.ndim != 2 or q.shape[1] != self.dim:
            raise ValueError(f"queries must be (B, {self.dim}) float32")
        t = ctypes.c_int64(0)
        _check(self.lib.hr_index_search_submit_host(self._h, _ptr(q), q.shape[0], int(k), int(notify_fd),
                                                    ctypes.byref(t)))
        return t.value

    def search_collect(self, ticket: int, B: int, k: int) -> tuple[np.ndarray, np.ndarray]:
        """(scores, rows) of a submitted asynchronous batch (waits if it is not done yet)."""
        s = np.empty((B, k), np.float32)
        r = np.empty((B, k), np.int64)
        _check(self.lib.hr_index_search_collect(self._h, int(ticket), _ptr(s), _ptr(r)))
        return s, r

    def search_poll(self, ticket: int) -> int:
        """State of a submitted asynchronous batch, without waiting: 0 running, 1 ready, 2 ready but its
        collect will run the exact fallback (a corpus pass: collect it off the event loop).  Raises
        BusyError while another call holds the handle."""
        st = ctypes.c_int(0)
        _check(self.lib.hr_index_search_poll(self._h, int(ticket), ctypes.byref(st)))
        return st.value

    def search_finalize(self, ticket: int) -> None:
        """Wait for a submitted batch's guard flags and run its exact fallback (no-op if already final)."""
        _check(self.lib.hr_index_search_finalize(self._h, int(ticket)))

    def host_us(self) -> dict:
        """Host time of the pipelined search: caller us per submit, busiest shard thread us per batch."""
        out = (ctypes.c_double * 3)()
        _check(self.lib.hr_index_host_us(self._h, out))
        return {"submit_us": out[0], "shard_thread_us": out[1], "batches": int(out[2])}

    def search_shard(self, q_ptr: int, B: int, k: int, kc: int, row_offset: int, cand_ptr: int, bound_ptr: int,
                     mask_ptr: int = 0, stream: int = 0, tail_stream: int | None = None,
                     q_ready_event: int = 0) -> None:
        """Per-shard exact top-kc.  With tail_stream (!= stream) the scan runs on `stream` and
        select/rescore on `tail_stream` (pipelined; outputs ready in tail_stream order).
        q_ready_event (raw hipEvent_t, pipelined only): the queries are ready once it completes,
        which lets a large shard prep the queries and run its SAMPLE pass early (see hiprag.h)."""
        if tail_stream is not None:
            _check(self.lib.hr_index_search_shard_async_ev(self._h, ctypes.c_void_p(q_ptr), int(B), int(k), int(kc),
                                                           ctypes.c_void_p(mask_ptr or None), int(row_offset),
                                                           ctypes.c_void_p(cand_ptr), ctypes.c_void_p(bound_ptr),
                                                           ctypes.c_void_p(stream or None),
                                                           ctypes.c_void_p(tail_stream or None),
                                                           ctypes.c_void_p(q_ready_event or None)))
            return
        _check(self.lib.hr_index_search_shard(self._h, ctypes.c_void_p(q_ptr), int(B), int(k), int(kc),
                                              ctypes.c_void_p(mask_ptr or None), int(row_offset),
                                              ctypes.c_void_p(cand_ptr), ctypes.c_void_p(bound_ptr),
                                              ctypes.c_void_p(stream or None)))

    def search_shard_collect(self, q_ptr: int, B: int, kth_ptr: int, cap: int, row_offset: int, cand_ptr: int,
                             bound_ptr: int, mask_ptr: int = 0, stream: int = 0) -> None:
        _check(self.lib.hr_index_search_shard_collect(self._h, ctypes.c_void_p(q_ptr), int(B), ctypes.c_void_p(kth_ptr),
                                                      int(cap), ctypes.c_void_p(mask_ptr or None), int(row_offset),
                                                      ctypes.c_void_p(cand_ptr), ctypes.c_void_p(bound_ptr),
                                                      ctypes.c_void_p(stream or None)))

    def search_shard_exact(self, q_ptr: int, B: int, m: int, row_offset: int, cand_ptr: int, mask_ptr: int = 0,
                           stream: int = 0) -> None:
        """Exact top-m of every query over this shard (the exhaustive pass), B*m sorted records with global rows."""
        _check(self.lib.hr_index_search_shard_exact(self._h, ctypes.c_void_p(q_ptr), int(B), int(m),
                                                    ctypes.c_void_p(mask_ptr or None), int(row_offset),
                                                    ctypes.c_void_p(cand_ptr), ctypes.c_void_p(stream or None)))

    def debug_approx(self, q: np.ndarray) -> tuple[np.ndarray, np.ndarray]:
        """(approximate MFMA scores B×n, error bound E per query) -- diagnostics."""
        q = np.ascontiguousarray(q, np.float32)
        n, _ = self.size()
        out = np.empty((q.shape[0], n), np.float32)
        e = np.empty(q.shape[0], np.float64)
        _check(self.lib.hr_index_debug_approx(self._h, _ptr(q), q.shape[0], _ptr(out), _ptr(e)))
        return out, e

    def last_candidates(self) -> tuple[int, int]:
        t, m = ctypes.c_int64(0), ctypes.c_int64(0)
        _check(self.lib.hr_index_last_candidates(self._h, ctypes.byref(t), ctypes.byref(m)))
        return t.value, m.value

    def stats(self) -> dict:
        """Cumulative diagnostics: main scan passes, guard failures (collect fallback), exhaustive passes."""
        out = (ctypes.c_int64 * 3)()
        _check(self.lib.hr_index_stats(self._h, out))
        return {"main_passes": out[0], "guard_failures": out[1], "exhaustive": out[2]}

    def set_q256(self, on: bool) -> None:
        """The 256-query FILTER for 129-256-query batches (default on; off: two 128-query FILTER launches)."""
        _check(self.lib.hr_index_set_q256(self._h, 1 if on else 0))

    def q256_launches(self) -> int:
        """256-query FILTER launches issued so far (hr_index_q256_launches)."""
        out = ctypes.c_int64(0)
        _check(self.lib.hr_index_q256_launches(self._h, ctypes.byref(out)))
        return out.value

    def wide_launches(self) -> int:
        """128-query FILTER launches issued so far (hr_index_wide_launches)."""
        out = ctypes.c_int64(0)
        _check(self.lib.hr_index_wide_launches(self._h, ctypes.byref(out)))
        return out.value

    def wave_tiles(self, cap: int = 1 << 16) -> np.ndarray:
        """Tiles each wave of the most recent k_scan FILTER launch scanned ([group][wave], hr_index_wave_tiles)."""
        out = np.zeros(cap, np.uint32)
        n = ctypes.c_int(0)
        _check(self.lib.hr_index_wave_tiles(self._h, _ptr(out), int(cap), ctypes.byref(n)))
        return out[: n.value].copy()

    def set_persist(self, mode: int) -> None:
        """Persistent FILTER of pipelined shard batches: 0 off, 1 shards of 4.2M-5.1M rows (default), 2 any size."""
        _check(self.lib.hr_index_set_persist(self._h, int(mode)))

    def set_cu_mask(self, cus) -> None:
        """Run this index's internal streams on the CUs listed in `cus` (None / empty: all CUs); see
        hr_index_set_cu_mask and cu_mask_words."""
        words = cu_mask_words(cus) if cus else np.zeros(0, np.uint32)
        _check(self.lib.hr_index_set_cu_mask(self._h, words.ctypes.data if len(words) else None, len(words)))

    def persist_close(self) -> None:
        """No further batch for now: a running persistent FILTER exits once through its batches."""
        _check(self.lib.hr_index_persist_close(self._h))

    def persist_stats(self) -> dict:
        """Persistent FILTER diagnostics: batches served, error word (0 = none), instances that ran."""
        out = (ctypes.c_int64 * 3)()
        _check(self.lib.hr_index_persist_stats(self._h, out))
        return {"batches": out[0], "error": out[1], "runs": out[2]}

    def persist_trace(self, n: int = 64) -> np.ndarray:
        """[epochs, 5] device stamps (us, from the first returned post) of the last n persistent batches: post,
        first / last workgroup start, first / last workgroup arrival."""
        out = np.zeros((max(0, int(n)), 5), np.float64)
        m = ctypes.c_int(0)
        _check(self.lib.hr_index_persist_trace(self._h, int(n), out.ctypes.data, ctypes.byref(m)))
        return out[: m.value].copy()

    def graph_replays(self) -> int:
        """hr_index_search calls answered by a captured HIP graph (hr_index_graph_replays)."""
        n = ctypes.c_int64(0)
        _check(self.lib.hr_index_graph_replays(self._h, ctypes.byref(n)))
        return n.value

    def set_scan_timing(self, every: int) -> None:
        """Record HIP events around every `every`-th main-pass scan (0 = off, the default)."""
        _check(self.lib.hr_index_set_scan_timing(self._h, int(every)))

    def take_scan_times(self, cap: int = 1 << 16) -> tuple[np.ndarray, np.ndarray]:
        """(sample_ms, filter_ms) of every main-pass scan since the previous harvest."""
        a = np.empty(cap, np.float32)
        b = np.empty(cap, np.float32)
        n = ctypes.c_int(0)
        _check(self.lib.hr_index_take_scan_times(self._h, _ptr(a), _ptr(b), int(cap), ctypes.byref(n)))
        return a[: n.value].copy(), b[: n.value].copy()

    def last_scan_ms(self) -> tuple[float, float]:
        a, b = ctypes.c_float(0), ctypes.c_float(0)
        _check(self.lib.hr_index_last_scan_ms(self._h, ctypes.byref(a), ctypes.byref(b)))
        return a.value, b.value

    # -- persistence
    def save(self, path: str) -> None:
        _check(self.lib.hr_index_save(self._h, os.fsencode(path)))

    @classmethod
    def load(cls, path: str, device: int = 0, dim: int | None = None, dtype: str | None = None,
             metric: str | None = None, devices: list[int] | None = None) -> "NativeIndex":
        L = load_library()
        h = ctypes.c_void_p()
        devs = [int(d) for d in devices] if devices else [int(device)]
        dev = (ctypes.c_int * len(devs))(*devs)
        _check(L.hr_index_load(os.fsencode(path), len(devs), dev, ctypes.byref(h)))
        d, dt, m, g = (ctypes.c_int(0) for _ in range(4))
        _check(L.hr_index_info(h, ctypes.byref(d), ctypes.byref(dt), ctypes.byref(m), ctypes.byref(g)))
        # the file's own shape (the dim / dtype / metric arguments are only checked against it)
        dtype_f = {0: "f32", 1: "bf16", 2: "f16"}[dt.value]
        metric_f = {0: "cosine", 1: "ip", 2: "l2"}[m.value]
        if (dim and int(dim) != d.value) or (dtype and DTYPES.get(dtype) != dt.value) or \
                (metric and METRICS.get(metric) != m.value):
            L.hr_index_destroy(h)
            raise ValueError(f"{path}: index is dim={d.value} dtype={dtype_f} metric={metric_f}, "
                             f"not dim={dim} dtype={dtype} metric={metric}")
        return cls(d.value, dtype_f, metric_f, devs[0], devices=devs, _handle=h)


def gen_rows_device(seed: int, row0: int, n: int, dim: int, out_ptr: int, stream: int = 0) -> None:
    """Synthetic corpus rows [row0, row0 + n) as fp32 into device memory (the hr_index_add_synthetic generator)."""
    _check(load_library().hr_gen_rows_device(int(seed), int(row0), int(n), int(dim), ctypes.c_void_p(out_ptr),
                                             ctypes.c_void_p(stream or None)))


def topk_records(in_ptr: int, B: int, m: int, out_ptr: int, seg_stride: int = 0, seg_off_ptr: int = 0,
                 stream: int = 0) -> None:
    """Exact top-m {score f64, id i64} records per segment, (score desc, id asc) (hr_topk_records)."""
    _check(load_library().hr_topk_records(ctypes.c_void_p(in_ptr), ctypes.c_void_p(seg_off_ptr or None),
                                          int(seg_stride), int(B), int(m), ctypes.c_void_p(out_ptr),
                                          ctypes.c_void_p(stream or None)))


def merge_candidates(device: int, cand_ptr: int, bounds_ptr: int, G: int, B: int, kc: int, k: int, scores_ptr: int,
                     rows_ptr: int, kth_ptr: int, fail_ptr: int, stream: int = 0, cand_rank_stride: int = 0,
                     bound_rank_stride: int = 0) -> None:
    """Merge G ranks' candidates; strides (bytes) default to the dense [G][B][kc] / [G][B] layouts."""
    L = load_library()
    if cand_rank_stride or bound_rank_stride:
        _check(L.hr_merge_candidates_strided(int(device), ctypes.c_void_p(cand_ptr), ctypes.c_void_p(bounds_ptr),
                                             int(cand_rank_stride or B * kc * 16), int(bound_rank_stride or B * 8),
                                             int(G), int(B), int(kc), int(k), ctypes.c_void_p(scores_ptr),
                                             ctypes.c_void_p(rows_ptr), ctypes.c_void_p(kth_ptr),
                                             ctypes.c_void_p(fail_ptr), ctypes.c_void_p(stream or None)))
        return
    _check(L.hr_merge_candidates(int(device), ctypes.c_void_p(cand_ptr), ctypes.c_void_p(bounds_ptr),
                                 int(G), int(B), int(kc), int(k), ctypes.c_void_p(scores_ptr),
                                 ctypes.c_void_p(rows_ptr), ctypes.c_void_p(kth_ptr),
                                 ctypes.c_void_p(fail_ptr), ctypes.c_void_p(stream or None)))


def merge_sorted(device: int, cand_ptr: int, G: int, B: int, m: int, k: int, scores_ptr: int, rows_ptr: int,
                 stream: int = 0, cand_rank_stride: int = 0) -> None:
    """Merge G ranks' sorted exact top-m lists (search_shard_exact records) into the top-k (hr_merge_sorted)."""
    _check(load_library().hr_merge_sorted(int(device), ctypes.c_void_p(cand_ptr), int(cand_rank_stride), int(G),
                                          int(B), int(m), int(k), ctypes.c_void_p(scores_ptr),
                                          ctypes.c_void_p(rows_ptr), ctypes.c_void_p(stream or None)))


def pool_normalize(hidden_ptr: int, dtype: str, mask_ptr: int, B: int, T: int, H: int, n_instr: int, out_ptr: int,
                   stream: int = 0) -> None:
    _check(load_library().hr_pool_normalize(ctypes.c_void_p(hidden_ptr), DTYPES[dtype], ctypes.c_void_p(mask_ptr),
                                            int(B), int(T), int(H), int(n_instr), ctypes.c_void_p(out_ptr),
                                            ctypes.c_void_p(stream or None)))


def pool_normalize_packed(hidden_ptr: int, dtype: str, cu_ptr: int, B: int, H: int, n_instr: int, out_ptr: int,
                          stream: int = 0) -> None:
    """K7 over packed hidden states (rows [cu[b], cu[b+1]) are sequence b; cu: B+1 int32 on the device)."""
    _check(load_library().hr_pool_normalize_packed(ctypes.c_void_p(hidden_ptr), DTYPES[dtype], ctypes.c_void_p(cu_ptr),
                                                   int(B), int(H), int(n_instr), ctypes.c_void_p(out_ptr),
                                                   ctypes.c_void_p(stream or None)))


def hash_words(data: bytes, offsets, first_id: int, span: int, cap: int = -1, cls_id: int = -1, sep_id: int = -1):
    """Host text kernel of the offline tokenizer (hr_hash_words): ASCII texts packed in `data` with int64
    `offsets` (n+1) -> (ids int64 flat, lengths int64 (n,)).  No GPU involved."""
    import numpy as np

    offsets = np.ascontiguousarray(offsets, dtype=np.int64)
    n = len(offsets) - 1
    cap_ids = len(data) + 2 * n + 1  # every token takes at least one byte
    ids = np.empty(cap_ids, np.int64)
    lengths = np.empty(max(n, 0), np.int64)
    _check(load_library().hr_hash_words(data, offsets.ctypes.data_as(ctypes.c_void_p), int(n), int(first_id),
                                        int(span), int(cap), int(cls_id), int(sep_id),
                                        ids.ctypes.data_as(ctypes.c_void_p), int(cap_ids),
                                        lengths.ctypes.data_as(ctypes.c_void_p)))
    return ids[:int(lengths.sum())], lengths


_ATTN_DT = {"bfloat16": "bf16", "float16": "f16"}


def attn_varlen(qkv, cu, B: int, nH: int, d: int, max_len: int, scale: float, out=None):
    """Short-sequence attention of a packed batch (hr_attn_varlen): qkv (N, 3 nH d) bf16 / f16 device tensor, cu
    (B + 1,) int32 device offsets -> (N, nH d).  Returns None where the kernel does not apply (d != 64, a sequence
    longer than 64 tokens, ...): the caller runs the flash varlen kernel instead."""
    import torch

    dt = _ATTN_DT.get(str(qkv.dtype).replace("torch.", ""))
    if dt is None or d != 64 or max_len > 64 or not qkv.is_contiguous():
        return None
    n = qkv.shape[0]
    out = out if out is not None else torch.empty((n, nH * d), dtype=qkv.dtype, device=qkv.device)
    rc = load_library().hr_attn_varlen(ctypes.c_void_p(qkv.data_ptr()), DTYPES[dt], ctypes.c_void_p(cu.data_ptr()),
                                       int(B), int(nH), int(d), int(max_len), float(scale),
                                       ctypes.c_void_p(out.data_ptr()),
                                       ctypes.c_void_p(torch.cuda.current_stream(qkv.device).cuda_stream))
    if rc == E_UNSUPPORTED:
        return None
    _check(rc)
    return out


def gelu_erf_(x):
    """In-place exact GELU of a bf16 / f16 device tensor (hr_gelu_erf); returns x, or None if it does not apply."""
    import torch

    dt = _ATTN_DT.get(str(x.dtype).replace("torch.", ""))
    if dt is None or not x.is_contiguous():
        return None
    rc = load_library().hr_gelu_erf(ctypes.c_void_p(x.data_ptr()), DTYPES[dt], x.numel(),
                                    ctypes.c_void_p(torch.cuda.current_stream(x.device).cuda_stream))
    if rc == E_UNSUPPORTED:
        return None
    _check(rc)
    return x


def add_layernorm(x, r, weight, bias, eps: float):
    """K8: LayerNorm(x + r) with affine weight/bias over the last dim, one fused HIP kernel (torch
    tensors on one device, same dtype, contiguous; runs on the current stream)."""
    import torch

    names = {torch.float32: "f32", torch.bfloat16: "bf16", torch.float16: "f16"}
    if x.dtype not in names or r.dtype != x.dtype or weight.dtype != x.dtype or bias.dtype != x.dtype:
        raise ValueError("add_layernorm: x, r, weight and bias must share one of f32 / bf16 / f16")
    if x.shape != r.shape or weight.shape != (x.shape[-1],) or bias.shape != (x.shape[-1],):
        raise ValueError("add_layernorm: shape mismatch")
    x, r = x.contiguous(), r.contiguous()
    out = torch.empty_like(x)
    H = x.shape[-1]
    _check(load_library().hr_add_layernorm(ctypes.c_void_p(x.data_ptr()), ctypes.c_void_p(r.data_ptr()),
                                           ctypes.c_void_p(weight.data_ptr()), ctypes.c_void_p(bias.data_ptr()),
                                           ctypes.c_void_p(out.data_ptr()), x.numel() // H, H, float(eps),
                                           DTYPES[names[x.dtype]],
                                           ctypes.c_void_p(torch.cuda.current_stream(x.device).cuda_stream)))
    return out

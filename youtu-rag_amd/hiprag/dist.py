"""Row-sharded multi-GPU search: one process per GPU, RCCL over xGMI for the merge.

The corpus is split into contiguous row ranges, one per rank (global row =
shard offset + local row).  Every rank scans its shard for the same replicated
query batch and produces, per query, its exact top-kc candidates (fp64 canonical
scores + global rows) and a bound on the score of every row it did NOT return.
One ``all_gather`` moves each rank's packed record -- B·kc 16-byte candidates followed by
its B bounds, 33 KB at B=64, kc=32 -- latency-bound, so exactly one collective per batch
and nothing else crosses xGMI; each rank then
merges the G·kc candidates on its own GPU with the same (score desc, row asc)
order and the same guard, so all ranks hold identical results.  Queries whose
guard fails (top-k not provably complete) are re-scanned in collect mode: every
shard returns all rows whose approximate score could still reach the k-th exact
score (a shard whose window overflows its buffer returns its exact top rows
instead), and a second merge is exact by construction.

Every k the single index serves is served here too (Chroma's ``n_results`` has no
cap, /root/reference/utu/rag/storage/implementations/chroma_store.py:118-120;
FAISS returns the exact top-k whatever the ties, faiss_store.py:148-176): a k above
the pipelined kc runs as one synchronous batch -- the scan with kc_for_k(k) up to
HR_MAX_K, above that every shard's exhaustive exact top-k (hr_index_search_shard_exact),
all-gathered and merged by rank (hr_merge_sorted).

Batches are pipelined at two levels.  On the GPU, each batch's scan runs on the caller's
stream over all but a few CUs, while the previous batch's select/rescore, all-gather and
merge run on a second ("tail") stream on the CUs left free -- the scan reads HBM as fast
on 224 CUs as on 256, so the tail costs no scan time.  On the host, ``submit`` enqueues a
whole batch (scan, tail, a non-blocking copy of the guard flags) and returns a ticket;
``finalize`` waits for that batch's flags only and runs the (rare) fallback.  With
``depth`` tickets in flight the host's per-batch work overlaps the GPU's.

The reference is single-process (SURVEY.md §2 "Parallelism strategies: none");
this module is the C1 collective of the SURVEY kernel inventory.
"""
from __future__ import annotations

import time

import numpy as np

from . import _native

def fallback_cap(G: int) -> int:
    """Rows per query and shard the collect fallback may return: 1024, bounded so the merge of
    G shards' records fits the merge kernel's LDS (G * cap <= 8192)."""
    return max(64, min(1024, 8192 // max(1, G)))


class _Done:
    """Ticket of a batch answered inside submit (k above the pipelined kc): finalize returns its outputs."""

    __slots__ = ("result",)

    def __init__(self, s_out, r_out):
        self.result = (s_out, r_out)


def _record_len(B: int, kc: int) -> int:
    """float64 words of one rank's packed all-gather record: B*kc {score, row} pairs, then B bounds."""
    return B * kc * 2 + B


def _record_views(rec, B: int, kc: int):
    """(cand (..., B, kc, 2), bound (..., B)) views of packed records rec (..., _record_len)."""
    n = B * kc * 2
    return rec[..., :n].view(*rec.shape[:-1], B, kc, 2), rec[..., n:n + B]


class RcclComm:
    """An RCCL communicator of the process group's ranks, called directly (ctypes, the librccl.so torch loaded) on
    the streams the exchange is ordered on -- the tail stream for the all-gather, the scan stream for a broadcast.

    Through torch.distributed an RCCL collective runs on the process group's own internal stream, joined to the
    caller's stream by an event each way; with GPU_MAX_HW_QUEUES = 4 that extra stream shares a hardware queue
    with the scan or tail streams, and the tail's all-gather then queues behind the next batch's FILTER launch:
    a 1.25M-row shard (the G = 8 per-rank step) ran 0.448-0.469 ms/step through it against 0.418 with the
    local copy, at world size 1, where the host work per step is only 0.09 ms (profiles/
    r04_rccl_world1_host_time.jsonl).  A direct ncclAllGather on the tail stream adds no stream.  The unique
    id goes to every rank with one broadcast over the process group; ncclCommInitRank is collective (every rank
    constructs this at the same point)."""

    def __init__(self, torch, dist, group, device, lib=None):
        """lib: the RCCL library (default: the librccl.so torch loaded); the CPU tests pass a ctypes-shaped stand-in
        that moves the bytes over gloo, so this G > 1 control flow runs without GPUs."""
        import ctypes
        import contextlib
        import os

        self.ct = ctypes
        if lib is None:
            lib = ctypes.CDLL(os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so"))
        self.lib = lib
        lib.ncclGetErrorString.restype = ctypes.c_char_p
        for f in ("ncclAllGather", "ncclBroadcast", "ncclCommInitRank", "ncclGetUniqueId", "ncclCommDestroy"):
            getattr(lib, f).restype = ctypes.c_int

        class _Uid(ctypes.Structure):
            _fields_ = [("internal", ctypes.c_char * 128)]

        self.rank = dist.get_rank(group)
        self.G = dist.get_world_size(group)
        uid = _Uid()
        if self.rank == 0:
            self._check(lib.ncclGetUniqueId(ctypes.byref(uid)))
        buf = torch.frombuffer(bytearray(bytes(uid)), dtype=torch.uint8).to(device)
        src = dist.get_global_rank(group, 0) if group is not None else 0
        dist.broadcast(buf, src, group=group)
        uid = _Uid.from_buffer_copy(bytes(buf.cpu().numpy().tobytes()))
        self.comm = ctypes.c_void_p()
        dev = torch.device(device)
        with torch.cuda.device(dev) if dev.type == "cuda" else contextlib.nullcontext():
            self._check(lib.ncclCommInitRank(ctypes.byref(self.comm), self.G, uid, self.rank))

    def _check(self, rc: int) -> None:
        if rc != 0:
            raise RuntimeError(f"RCCL error {rc}: {self.lib.ncclGetErrorString(rc).decode()}")

    def all_gather(self, out_ptr: int, in_ptr: int, nbytes: int, stream: int) -> None:
        c = self.ct
        self._check(self.lib.ncclAllGather(c.c_void_p(in_ptr), c.c_void_p(out_ptr), c.c_size_t(nbytes), 1,  # uint8
                                           self.comm, c.c_void_p(stream)))

    def broadcast(self, ptr: int, nbytes: int, root: int, stream: int) -> None:
        c = self.ct
        self._check(self.lib.ncclBroadcast(c.c_void_p(ptr), c.c_void_p(ptr), c.c_size_t(nbytes), 1, root,
                                           self.comm, c.c_void_p(stream)))

    def close(self) -> None:
        if self.comm:
            self._check(self.lib.ncclCommDestroy(self.comm))
            self.comm = self.ct.c_void_p()


class _Slot:
    def __init__(self, torch, device, G, B, kc, pinned, gather: bool):
        f64 = dict(dtype=torch.float64, device=device)
        self.rec = torch.empty((_record_len(B, kc),), **f64)  # this rank's packed record
        # the gathered records (G > 1, or G = 1 with the collective forced); else the merge reads rec itself
        self.rec_all = torch.empty((G, _record_len(B, kc)), **f64) if gather else None
        self.kth = torch.empty((B,), **f64)
        self.fail = torch.empty((B,), dtype=torch.int32, device=device)
        self.fail_h = torch.empty((B,), dtype=torch.int32, pin_memory=pinned)
        self.event = torch.cuda.Event() if pinned else None
        self.ticket = None  # (q, k, s_out, r_out, mask_ptr, B) while in flight
        self._views: dict = {}
        self._qbuf = None
        self.q_event = torch.cuda.Event() if pinned else None

    def qbuf(self, shape, dtype):
        """This slot's query buffer for broadcast batches (the slot owns it until finalize)."""
        import torch

        if self._qbuf is None or self._qbuf.shape != shape or self._qbuf.dtype != dtype:
            self._qbuf = torch.empty(shape, dtype=dtype, device=self.kth.device)
        return self._qbuf

    def views(self, B: int, kc: int):
        """(L, record, cand, bound) of a B-query batch -- cached: views cost host time every batch."""
        v = self._views.get(("r", B))
        if v is None:
            L = _record_len(B, kc)
            rec = self.rec[:L]
            v = self._views[("r", B)] = (L, rec, *_record_views(rec, B, kc))
        return v

    def views_all(self, B: int, kc: int, G: int):
        """(rec_all, cand_all, bound_all, kth, fail) of a B-query batch over G ranks (cached)."""
        v = self._views.get(("a", B))
        if v is None:
            L, rec = self.views(B, kc)[:2]
            rec_all = rec.view(1, L) if self.rec_all is None else self.rec_all.view(-1)[: G * L].view(G, L)
            v = self._views[("a", B)] = (rec_all, *_record_views(rec_all, B, kc), self.kth[:B], self.fail[:B])
        return v


class ShardedSearch:
    """Distributed exact top-k over a row-sharded index (torch.distributed group)."""

    def __init__(self, index, row_offset: int, max_batch: int, kc: int | None = None, group=None,
                 device=None, depth: int = 2, max_k: int = 16, overlap: bool = True, force_collective: bool = False,
                 rccl_lib=None):
        """force_collective: run the exchange (all-gather of the packed records, broadcast of src_rank
        batches) through the process group even at world size 1, where it is otherwise a local copy --
        so a one-GPU box executes the RCCL branch an 8-GPU node runs (bench.py --collective).
        rccl_lib: take the direct-RCCL branch (RcclComm) with this library object whatever the backend (CPU tests of
        the G > 1 control flow with a stand-in library)."""
        import torch
        import torch.distributed as dist

        self.torch, self.dist = torch, dist
        self.index = index
        self.row_offset = int(row_offset)
        self.group = group
        self.G = dist.get_world_size(group) if dist.is_initialized() else 1
        if force_collective and not dist.is_initialized():
            raise ValueError("force_collective needs an initialised process group")
        self.collective = self.G > 1 or bool(force_collective)  # the exchange goes through the process group
        self.fallback_queries = 0  # queries whose guard failed (collect fallback), cumulative
        self.exact_queries = 0  # queries answered by the shards' exhaustive exact pass (large k), cumulative
        self.collective_calls = {"all_gather": 0, "broadcast": 0}  # exchanges through the process group's ranks
        self.wait_s = 0.0  # host time blocked on guard flags in finalize (the rest of a submit is host work)
        # candidates per shard per query: kc_for_k(max_k) keeps the guard's margin for every k <= max_k
        # (16 -> kc 32, one row part); a larger k up to kc is served, with a thinner margin
        self.kc = int(kc) if kc is not None else _native.kc_for_k(max_k, int(getattr(index, "dim", 0)))
        self.max_batch = int(max_batch)
        self.device = device if device is not None else torch.device("cuda", torch.cuda.current_device())
        pinned = self.device.type == "cuda"
        self._dev_index = self.device.index if self.device.index is not None else 0
        self.slots = [_Slot(torch, self.device, self.G, self.max_batch, self.kc, pinned, self.collective)
                      for _ in range(max(1, depth))]
        self._next = 0
        # tail stream: select/rescore, all-gather, merge and the flag copy of each batch
        self.tail = torch.cuda.Stream(self.device) if (overlap and pinned) else None
        # RCCL itself on the tail / scan streams (RcclComm) when the group is nccl; gloo (CPU tests) goes
        # through torch.distributed with host staging
        self.backend = dist.get_backend(group) if self.collective else None
        if self.collective and rccl_lib is not None:
            self.rccl = RcclComm(torch, dist, group, self.device, lib=rccl_lib)
        else:
            self.rccl = RcclComm(torch, dist, group, self.device) if (self.collective and self.backend == "nccl"
                                                                       and pinned) else None
        self.transport = ("rccl (direct, on the tail stream)" if self.rccl is not None else
                          f"torch.distributed ({self.backend})" if self.collective else "local copy")

    # hooks (overridden in CPU tests of the orchestration logic)
    def _stream(self) -> int:
        # the raw handle of the current stream without torch.cuda.current_stream's Python layers (called
        # several times per batch; on a small collection the host submission bounds the step)
        raw = getattr(self.torch._C, "_cuda_getCurrentRawStream", None)
        if raw is not None:
            return raw(self._dev_index)
        return self.torch.cuda.current_stream(self.device).cuda_stream

    def _merge(self, cand_all, bound_all, G, B, kc, k, s_out, r_out, kth, fail):
        # cand_all (G, B, kc, 2) / bound_all (G, B): views into packed per-rank records (rank stride
        # = stride(0)); the kernel reads them in place
        _native.merge_candidates(self.device.index or 0, cand_all.data_ptr(), bound_all.data_ptr(), G, B, kc, k,
                                 s_out.data_ptr(), r_out.data_ptr(), kth.data_ptr(), fail.data_ptr(), self._stream(),
                                 cand_rank_stride=cand_all.stride(0) * 8, bound_rank_stride=bound_all.stride(0) * 8)

    def _shard_search(self, q, k, cand, bound, mask_ptr, q_ready=None, kc=None):
        """This shard's exact top-kc candidates and bound.  kc None: the pipelined batch (self.kc, scan + tail
        streams); else a synchronous scan with that kc on the current stream (k above the pipelined kc)."""
        if kc is not None:
            self.index.search_shard(q.data_ptr(), q.shape[0], k, kc, self.row_offset, cand.data_ptr(),
                                    bound.data_ptr(), mask_ptr=mask_ptr, stream=self._stream())
            return
        tail = self.tail.cuda_stream if self.tail is not None else None
        ev = q_ready.cuda_event if (q_ready is not None and tail is not None) else 0
        self.index.search_shard(q.data_ptr(), q.shape[0], k, self.kc, self.row_offset, cand.data_ptr(),
                                bound.data_ptr(), mask_ptr=mask_ptr, stream=self._stream(), tail_stream=tail,
                                q_ready_event=ev)

    def _shard_exact(self, q, m, cand, mask_ptr):
        """This shard's exact top-m of every query (exhaustive pass): cand (B, m, 2) float64 records, sorted."""
        self.index.search_shard_exact(q.data_ptr(), q.shape[0], m, self.row_offset, cand.data_ptr(),
                                      mask_ptr=mask_ptr, stream=self._stream())

    def _merge_sorted(self, cand_all, G, B, m, k, s_out, r_out):
        # cand_all (G, B, m, 2): every rank's sorted exact lists, rank stride = stride(0)
        _native.merge_sorted(self.device.index or 0, cand_all.data_ptr(), G, B, m, k, s_out.data_ptr(),
                             r_out.data_ptr(), self._stream(), cand_rank_stride=cand_all.stride(0) * 8)

    def _shard_collect(self, q, kth, cap, cand, bound, mask_ptr):
        self.index.search_shard_collect(q.data_ptr(), q.shape[0], kth.data_ptr(), cap, self.row_offset,
                                        cand.data_ptr(), bound.data_ptr(), mask_ptr=mask_ptr, stream=self._stream())

    def _all_gather(self, out, inp):
        if not self.collective:
            out[0].copy_(inp)
        else:
            self.collective_calls["all_gather"] += 1
            if self.rccl is not None:  # out (G, L) contiguous, rank r's record at row r
                self._on_tail(lambda st: self.rccl.all_gather(out.data_ptr(), inp.data_ptr(),
                                                              inp.numel() * inp.element_size(), st))
                return
            # output as the rank-concatenation along dim 0 (accepted by RCCL and gloo alike)
            flat = out.view(self.G * inp.shape[0], *inp.shape[1:])
            if out.is_cuda and self.backend != "nccl":
                # gloo (tests: several ranks sharing one GPU) gathers host tensors
                tmp = flat.cpu()
                self.dist.all_gather_into_tensor(tmp, inp.cpu().contiguous(), group=self.group)
                flat.copy_(tmp)
            else:
                self.dist.all_gather_into_tensor(flat, inp.contiguous(), group=self.group)

    def _on_tail(self, issue):
        """Issue a direct RCCL call on the tail stream: every collective of the communicator then runs in ONE
        stream's order on every rank (two streams could interleave two collectives differently on different ranks
        and deadlock).  From another stream (the fallback's gather, a broadcast before the scan) the tail waits for
        it first and it waits for the tail after -- rare paths; the per-batch gather is issued on the tail."""
        torch = self.torch
        if self.tail is None:  # (no tail stream: one stream's order already)
            issue(self._stream())
            return
        cur = torch.cuda.current_stream(self.device)
        if cur == self.tail:
            issue(self._stream())
            return
        self.tail.wait_stream(cur)
        issue(self.tail.cuda_stream)
        cur.wait_stream(self.tail)

    # the search
    def _broadcast(self, t, src: int):
        self.collective_calls["broadcast"] += 1
        if self.rccl is not None:  # src: a global rank; the communicator's ranks are the group's
            root = self.dist.get_group_rank(self.group, src) if self.group is not None else src
            self._on_tail(lambda st: self.rccl.broadcast(t.data_ptr(), t.numel() * t.element_size(), root, st))
            return
        if t.is_cuda and self.backend != "nccl":  # gloo (tests): host staging
            h = t.cpu()
            self.dist.broadcast(h, src, group=self.group)
            t.copy_(h)
        else:
            self.dist.broadcast(t, src, group=self.group)

    def submit(self, q, k: int, s_out=None, r_out=None, mask_ptr: int = 0, q_ready=None, src_rank: int | None = None):
        """Enqueue one batch; returns a ticket for finalize().  q: (B, dim) float32 device tensor,
        identical on every rank.  q_ready: optional recorded torch.cuda.Event after which q (and
        the mask) are ready; then a large shard preps the queries and runs its SAMPLE pass beside
        the previous batch's FILTER scan instead of after it.  Without it the queries are taken to
        be ready in the current stream's order."""
        torch = self.torch
        B = int(q.shape[0])
        k = int(k)
        if B > self.max_batch:
            raise ValueError(f"batch {B} > max_batch {self.max_batch}")
        if k < 1:
            raise ValueError("k must be >= 1")
        if k > self.kc:
            return self._submit_beyond_kc(q, k, s_out, r_out, mask_ptr, src_rank)
        slot = self.slots[self._next]
        self._next = (self._next + 1) % len(self.slots)
        if slot.ticket is not None:
            self.finalize(slot)
        q = q.contiguous()
        if src_rank is not None and self.collective:
            # the batch arrives on one rank: ONE broadcast (RCCL over xGMI, 4*B*dim bytes) on the scan
            # stream puts it on every rank before the scan (queries sent with a broadcast)
            qb = slot.qbuf(q.shape, q.dtype)
            qb.copy_(q)
            self._broadcast(qb, src_rank)
            q = qb
            if q_ready is not None:  # the early SAMPLE must wait for the broadcast, not the caller's event
                q_ready = slot.q_event
                q_ready.record()
        s_out = s_out if s_out is not None else torch.empty((B, k), dtype=torch.float32, device=self.device)
        r_out = r_out if r_out is not None else torch.empty((B, k), dtype=torch.int64, device=self.device)
        L, rec, cand, bound = slot.views(B, self.kc)
        self._shard_search(q, k, cand, bound, mask_ptr, q_ready)
        if self.tail is not None:
            # The caller's earlier writes to s_out/r_out (allocation, earlier use) were enqueued on its
            # stream before this batch's FILTER scan, and the native search makes the tail stream wait
            # for that scan (search_shard with tail_stream), so no torch wait_stream is needed here: its
            # event record would cost a ~6 us bubble on the scan stream every batch.
            with torch.cuda.stream(self.tail):
                self._exchange_and_merge(slot, rec, L, B, k, s_out, r_out)
        else:
            self._exchange_and_merge(slot, rec, L, B, k, s_out, r_out)
        slot.ticket = (q, k, s_out, r_out, mask_ptr, B)
        return slot

    def _exchange_and_merge(self, slot, rec, L, B, k, s_out, r_out):
        torch = self.torch
        rec_all, cand_all, bound_all, kth, fail = slot.views_all(B, self.kc, self.G)
        if self.collective:  # ONE collective per batch: every rank's packed record
            self._all_gather(rec_all, rec)
        self._merge(cand_all, bound_all, self.G, B, self.kc, k, s_out, r_out, kth, fail)
        if slot.event is not None:
            # the flags to pinned memory by a library copy, not torch's non_blocking copy_: torch's pinned-memory
            # allocator would record this (possibly caller-owned, e.g. CU-masked) stream and use it again when
            # fail_h is freed, after the caller may have destroyed it
            _native.memcpy_async(slot.fail_h.data_ptr(), fail.data_ptr(), B * 4, self._stream())
            slot.event.record(torch.cuda.current_stream(self.device))
        else:
            slot.fail_h[:B].copy_(fail)

    def finalize(self, slot) -> tuple:
        """Wait for a submitted batch's guard flags (only those) and run its fallback if needed."""
        if isinstance(slot, _Done):
            return slot.result
        if slot.ticket is None:
            raise ValueError("ticket already finalized")
        q, k, s_out, r_out, mask_ptr, B = slot.ticket
        slot.ticket = None
        if slot.event is not None:
            t0 = time.perf_counter()
            slot.event.synchronize()
            self.wait_s += time.perf_counter() - t0
        failed = self._failed_queries(slot, B)
        if len(failed):
            self.fallback_queries += len(failed)
            self._fallback(q, k, failed, slot.kth[:B], s_out, r_out, mask_ptr)
        return s_out, r_out

    def _failed_queries(self, slot, B: int):
        """Indices of the batch's queries whose guard failed (hook: tests force the fallback)."""
        return np.nonzero(slot.fail_h[:B].numpy())[0]

    def close(self):
        """Finalize what is in flight and release the direct RCCL communicator (every rank, before the process
        group is destroyed)."""
        self.finalize_all()
        if self.rccl is not None:
            if self.device.type == "cuda":
                self.torch.cuda.synchronize(self.device)
            self.rccl.close()
            self.rccl = None

    def finalize_all(self):
        for i in range(len(self.slots)):
            slot = self.slots[(self._next + i) % len(self.slots)]
            if slot.ticket is not None:
                self.finalize(slot)
        close = getattr(self.index, "persist_close", None)
        if close is not None:  # no batch behind these: a running persistent FILTER may exit now
            close()

    def search(self, q, k: int, s_out=None, r_out=None, mask_ptr: int = 0, src_rank: int | None = None):
        """Synchronous search of one batch.  Returns (scores, rows) device tensors.  src_rank: the batch
        is only valid on that rank and is broadcast first (other ranks pass a tensor of the same shape)."""
        self.finalize_all()
        return self.finalize(self.submit(q, k, s_out, r_out, mask_ptr, src_rank=src_rank))

    def _submit_beyond_kc(self, q, k, s_out, r_out, mask_ptr, src_rank):
        """A batch with k above the pipelined kc, answered synchronously (the batches in flight first, so every
        rank issues its collectives in the same order): the scan with kc_for_k(k) while that fits the scan
        (k <= HR_MAX_K), else every shard's exhaustive exact top-k.  Returns a finished ticket."""
        torch = self.torch
        self.finalize_all()
        q = q.contiguous()
        if src_rank is not None and self.collective:
            qb = torch.empty_like(q)
            qb.copy_(q)
            self._broadcast(qb, src_rank)
            q = qb
        B = int(q.shape[0])
        s_out = s_out if s_out is not None else torch.empty((B, k), dtype=torch.float32, device=self.device)
        r_out = r_out if r_out is not None else torch.empty((B, k), dtype=torch.int64, device=self.device)
        kc2 = _native.kc_for_k(k, int(getattr(self.index, "dim", 0) or 0))
        if k <= _native.HR_MAX_K and k <= kc2 <= _native.HR_MAX_KC and self.G * kc2 <= 8192:
            f64 = dict(dtype=torch.float64, device=self.device)
            L = _record_len(B, kc2)
            rec = torch.empty((L,), **f64)
            cand, bound = _record_views(rec, B, kc2)
            self._shard_search(q, k, cand, bound, mask_ptr, kc=kc2)
            rec_all = torch.empty((self.G, L), **f64) if self.collective else rec.view(1, L)
            if self.collective:
                self._all_gather(rec_all, rec)
            cand_all, bound_all = _record_views(rec_all, B, kc2)
            kth = torch.empty((B,), **f64)
            fail = torch.empty((B,), dtype=torch.int32, device=self.device)
            self._merge(cand_all, bound_all, self.G, B, kc2, k, s_out, r_out, kth, fail)
            failed = np.nonzero(fail.cpu().numpy())[0]
            if len(failed):
                self.fallback_queries += len(failed)
                self._fallback(q, k, failed, kth, s_out, r_out, mask_ptr)
        else:
            self._exact(q, k, np.arange(B), s_out, r_out, mask_ptr)
        return _Done(s_out, r_out)

    def _exact(self, q, k, which, s_out, r_out, mask_ptr):
        """Queries `which` of the batch answered by every shard's exhaustive exact top-k: one all-gather of the
        sorted lists, then the rank merge (complete by construction: a row no shard returned has k rows of its
        own shard ahead of it)."""
        torch = self.torch
        idx = torch.as_tensor(np.asarray(which, np.int64), device=self.device)
        qf = q[idx].contiguous()
        Bf = len(which)
        rec = torch.empty((Bf, k, 2), dtype=torch.float64, device=self.device)
        self._shard_exact(qf, k, rec, mask_ptr)
        if self.collective:
            rec_all = torch.empty((self.G, Bf, k, 2), dtype=torch.float64, device=self.device)
            self._all_gather(rec_all, rec)
        else:
            rec_all = rec.unsqueeze(0)
        s2 = torch.empty((Bf, k), dtype=torch.float32, device=self.device)
        r2 = torch.empty((Bf, k), dtype=torch.int64, device=self.device)
        self._merge_sorted(rec_all, self.G, Bf, k, k, s2, r2)
        s_out[idx] = s2
        r_out[idx] = r2
        self.exact_queries += Bf

    def _fallback(self, q, k, failed, kth, s_out, r_out, mask_ptr):
        """Collect re-scan of the queries whose guard failed.  Each shard's window is complete (a window larger
        than the buffer returns that shard's exact top-cap rows), so with k <= cap the merge is exact; k above
        the cap goes to the exhaustive pass."""
        torch = self.torch
        Bf, cap = len(failed), fallback_cap(self.G)
        if k > cap:
            self._exact(q, k, failed, s_out, r_out, mask_ptr)
            return
        idx = torch.as_tensor(failed, device=self.device)
        qf = q[idx].contiguous()
        kf = kth[idx].contiguous()
        L = _record_len(Bf, cap)
        rec = torch.empty((L,), dtype=torch.float64, device=self.device)
        cand, bound = _record_views(rec, Bf, cap)
        self._shard_collect(qf, kf, cap, cand, bound, mask_ptr)
        rec_all = torch.empty((self.G, L), dtype=torch.float64, device=self.device)
        self._all_gather(rec_all, rec)
        cand_all, bound_all = _record_views(rec_all, Bf, cap)
        s2 = torch.empty((Bf, k), dtype=torch.float32, device=self.device)
        r2 = torch.empty((Bf, k), dtype=torch.int64, device=self.device)
        kth2 = torch.empty((Bf,), dtype=torch.float64, device=self.device)
        fail2 = torch.empty((Bf,), dtype=torch.int32, device=self.device)
        self._merge(cand_all, bound_all, self.G, Bf, cap, k, s2, r2, kth2, fail2)
        s_out[idx] = s2
        r_out[idx] = r2
        still = np.nonzero(fail2.cpu().numpy())[0]
        if len(still):  # (a shard reported an incomplete window: the exhaustive pass settles it; same on every rank)
            self._exact(q, k, np.asarray(failed)[still], s_out, r_out, mask_ptr)

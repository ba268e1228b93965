"""Oracle-backed stand-in for hiprag._native.NativeIndex -- CPU tests of the HOST logic only.

It lets the store/retriever/distributed orchestration be tested without a GPU; it is
injected explicitly (``index_factory=``) and never reachable from the product path.
"""
import numpy as np

import oracle
from oracle import ref_numpy as R


class OracleIndex:
    def __init__(self, dim, dtype="bf16", metric="cosine", device=0):
        self.dim, self.dtype, self.metric = dim, dtype, metric
        self.rows = np.zeros((0, dim), np.float32 if dtype == "f32" else np.uint16)
        self.live = np.zeros(0, bool)
        self.searches = 0

    def reserve(self, n):
        pass

    def add(self, x):
        x = np.asarray(x, np.float32)
        first = len(self.rows)
        self.rows = np.concatenate([self.rows, R.process_rows(x, self.metric, self.dtype)])
        self.live = np.concatenate([self.live, np.ones(len(x), bool)])
        return first

    def remove(self, rows):
        self.live[np.asarray(rows)] = False

    def size(self):
        return len(self.rows), int(self.live.sum())

    def get_rows(self, rows):
        return R.dequantize(self.rows[np.asarray(rows)], self.dtype)

    def search(self, q, k, mask=None):
        self.searches += 1
        q = np.asarray(q, np.float32)
        if q.ndim == 1:
            q = q[None]
        allowed = self.live.copy()
        if mask is not None and len(np.asarray(mask).reshape(-1)) * 64 < len(self.rows):
            raise ValueError("row mask shorter than the index")  # as hiprag._native.NativeIndex.search
        if mask is not None:
            bits = np.unpackbits(np.asarray(mask, np.uint64).view(np.uint8), bitorder="little")[: len(allowed)]
            allowed &= bits.astype(bool)
        s, r = oracle.c_search(self.rows, self.dtype, R.process_queries(q, self.metric), k,
                               oracle.mask_from_bool(allowed), nthreads=2, metric=self.metric)
        return s.astype(np.float32), r

    def close(self):
        pass

    # persistence (the C ABI writes <path>.tmp then renames; the fake does the same)
    def save(self, path):
        tmp = path + ".tmp"
        with open(tmp, "wb") as f:
            np.savez(f, rows=self.rows, live=self.live, dim=self.dim, dtype=self.dtype, metric=self.metric)
        import os

        os.replace(tmp, path)

    @classmethod
    def load(cls, path, dim=None, dtype=None, metric=None):
        with np.load(path, allow_pickle=False) as z:
            idx = cls(int(z["dim"]), str(z["dtype"]), str(z["metric"]))
            idx.rows, idx.live = z["rows"].copy(), z["live"].copy()
        return idx


class AsyncOracleIndex(OracleIndex):
    """OracleIndex with the asynchronous host-query entry point of NativeIndex (search_submit_host /
    search_collect): results are computed at submit, and the completion count is written to the caller's
    eventfd from a timer thread after `delay` seconds -- the GPU's host function, simulated.  At most two
    batches in flight, like the library, and like the library (hr_index_search_collect) a collect returns only
    once that batch's notification has been written: the caller may close the fd right after."""

    def __init__(self, *a, delay=0.002, **kw):
        super().__init__(*a, **kw)
        self.delay, self.tickets, self.next_ticket, self.busy = delay, {}, 1, False
        self.needs_fallback: set = set()  # tickets whose collect would run the exact fallback (poll -> 2)
        self.collected: list = []
        self.devices = [0]
        self.notified: dict = {}  # ticket -> threading.Event set once its eventfd write is done

    def search_submit_host(self, q, k, notify_fd=-1):
        import os
        import threading

        import hiprag._native as N

        if self.busy or len(self.tickets) >= 2:  # the library: any free slot of two, else HR_E_BUSY
            raise N.BusyError(N.E_BUSY, "handle busy")
        if self.live.sum() == 0:
            raise NotImplementedError("empty index")
        t = self.next_ticket
        self.next_ticket += 1
        self.tickets[t] = self.search(q, k)
        if notify_fd >= 0:
            done = self.notified[t] = threading.Event()

            def fire():
                try:
                    os.eventfd_write(notify_fd, 1)
                finally:
                    done.set()

            threading.Timer(self.delay, fire).start()
        return t

    def search_poll(self, ticket):
        import hiprag._native as N

        if self.busy:
            raise N.BusyError(N.E_BUSY, "handle busy")
        if ticket not in self.tickets:
            raise ValueError("unknown or collected ticket")
        return 2 if ticket in self.needs_fallback else 1

    def search_collect(self, ticket, B, k):
        ev = self.notified.pop(ticket, None)
        if ev is not None and not ev.wait(10):  # the library waits for its notify host function the same way
            raise RuntimeError("notification never written")
        self.needs_fallback.discard(ticket)
        self.collected.append(ticket)
        return self.tickets.pop(ticket)

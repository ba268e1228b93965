"""GPU: the persistent FILTER (hr_persist.hip) -- pipelined shard batches streamed by one long-lived launch.

Every batch goes through ShardedSearch (the bench's and the multi-GPU path: early SAMPLE on the pre stream, tail
stream, two Python slots) with queries ready by event, and is checked against the CPU oracle: consecutive batches
use different queries and rotate through the three device workspaces, so a stale query tile, floor or key table in
any slot would change ids.  Also: the instance's idle exit and relaunch (a host gap longer than its 300 us timeout),
other kinds of search between persistent batches (masked, synchronous, the collect fallback), a mutation between
batches (quiesce + reconfigure), fp32 / f16 rows, and mode 0 (per-batch launches) giving the same answers.
The default mode takes the persistent FILTER only for 4.2M-5.1M-row shards (where it measured faster); these
600k-row cases force it with mode 2 (the same kernel and hand-offs; bench.py --rows 5000000 runs the default).
"""
import time

import numpy as np
import pytest

import oracle
from oracle import ref_numpy as R

pytestmark = pytest.mark.gpu

N, DIM, B, K = 600_000, 256, 64, 10  # 18.75k tiles: above the early-SAMPLE floor (16k tiles), 2.3k units per instance


@pytest.fixture(scope="module")
def native():
    from hiprag import _native

    _native.load_library()
    return _native


def _queries(seed, n, dim, nb, rng):
    from hiprag import synth

    out = []
    for i in range(nb):
        if i % 2 == 0:
            q, _ = synth.planted_queries(seed, n, dim, B, qseed=500 + i)
        else:
            q = rng.standard_normal((B, dim)).astype(np.float32)
        out.append(q.astype(np.float32))
    return np.stack(out)


def _run(idx, qs, k, gaps=(), q_ready=True):
    import torch

    from hiprag.dist import ShardedSearch

    dev = torch.device("cuda", 0)
    qd = torch.from_numpy(qs).to(dev)
    ready = torch.cuda.Event()
    ready.record()
    ss = ShardedSearch(idx, 0, max_batch=B, device=dev, max_k=k)
    s = torch.empty((len(qs), B, k), dtype=torch.float32, device=dev)
    r = torch.empty((len(qs), B, k), dtype=torch.int64, device=dev)
    for i in range(len(qs)):
        if i in gaps:
            torch.cuda.synchronize()
            time.sleep(0.005)  # longer than the instance's idle timeout: it exits, the next batch relaunches
        ss.submit(qd[i], k, s_out=s[i], r_out=r[i], q_ready=ready if q_ready else None)
    ss.finalize_all()
    torch.cuda.synchronize()
    return s.cpu().numpy(), r.cpu().numpy()


def _check(s, r, s_ref, r_ref):
    np.testing.assert_array_equal(r, r_ref)
    np.testing.assert_array_equal(s, s_ref.astype(np.float32))


@pytest.mark.parametrize("dtype,metric", [("bf16", "cosine"), ("f16", "cosine"), ("f32", "cosine"), ("bf16", "ip")])
def test_persist_batches_vs_oracle(native, dtype, metric):
    rng = np.random.default_rng(7)
    idx = native.NativeIndex(DIM, dtype, metric)
    try:
        idx.reserve(N)
        idx.add_synthetic(3, 0, N)
        idx.set_persist(2)
        stored = oracle.c_build_synthetic(3, 0, N, DIM, dtype, metric)
        qs = _queries(3, N, DIM, 10, rng)
        b0 = idx.persist_stats()["batches"]
        s, r = _run(idx, qs, K, gaps=(6,))
        st = idx.persist_stats()
        assert st["error"] == 0
        assert st["batches"] - b0 == len(qs)  # every batch went through the persistent FILTER
        for i in range(len(qs)):
            _check(s[i], r[i], *oracle.c_search(stored, dtype, R.process_queries(qs[i], metric), K, metric=metric))
        # mode 0 (one FILTER launch per batch) gives the same answers
        idx.set_persist(0)
        s0, r0 = _run(idx, qs[:4], K)
        np.testing.assert_array_equal(r0, r[:4])
        np.testing.assert_array_equal(s0, s[:4])
        assert idx.persist_stats()["batches"] == st["batches"]
    finally:
        idx.close()


def test_persist_interleaved_with_other_searches_and_mutations(native):
    """Between persistent batches: a synchronous search, a masked pipelined batch (not persistent), the collect
    fallback of a batch whose guard fails (100 duplicate rows > kc), removes and an add (the instance quiesces, the
    workspaces are re-configured for the new row count) -- every answer identical to the oracle."""
    import torch

    from hiprag.dist import ShardedSearch

    rng = np.random.default_rng(11)
    raw = R.gen_rows(5, 0, N, DIM)
    dups = np.sort(rng.choice(N, 100, replace=False))
    raw[dups] = raw[dups[0]]
    idx = native.NativeIndex(DIM, "bf16", "cosine")
    try:
        idx.add(raw)
        idx.set_persist(2)
        stored = R.process_rows(raw, "cosine", "bf16")
        live = np.ones(N, bool)
        dev = torch.device("cuda", 0)
        ss = ShardedSearch(idx, 0, max_batch=B, device=dev, max_k=K)
        ready = torch.cuda.Event()

        def batch(q, mask=None):
            qd = torch.from_numpy(q).to(dev)
            ready.record()
            s = torch.empty((B, K), dtype=torch.float32, device=dev)
            r = torch.empty((B, K), dtype=torch.int64, device=dev)
            mptr = 0
            if mask is not None:
                md = torch.from_numpy(oracle.mask_from_bool(mask).view(np.int64)).to(dev)
                mptr = md.data_ptr()
            t = ss.submit(qd, K, s_out=s, r_out=r, q_ready=ready, mask_ptr=mptr)
            return t, s, r, q, mask, (qd, md if mask is not None else None)

        def check(item):
            t, s, r, q, mask, _ = item
            ss.finalize(t)
            allowed = live if mask is None else (live & mask)
            s_ref, r_ref = oracle.c_search(stored, "bf16", R.process_queries(q, "cosine"), K,
                                           oracle.mask_from_bool(allowed))
            _check(s.cpu().numpy(), r.cpu().numpy(), s_ref, r_ref)

        q_plain = [rng.standard_normal((B, DIM)).astype(np.float32) for _ in range(6)]
        q_dup = q_plain[0].copy()
        q_dup[:2] = raw[dups[0]]  # these two need the collect fallback (and then the exhaustive pass)
        sel = rng.random(N) < 0.5
        b0 = idx.persist_stats()["batches"]
        a = batch(q_plain[1])
        b = batch(q_dup)
        check(a)
        c = batch(q_plain[2], mask=sel)  # masked: one FILTER launch of its own
        check(b)
        d = batch(q_plain[3])
        check(c)
        check(d)
        s_sync, r_sync = idx.search(q_plain[4], K)  # synchronous search in between
        _check(s_sync, r_sync, *oracle.c_search(stored, "bf16", R.process_queries(q_plain[4], "cosine"), K))
        e = batch(q_plain[5])
        check(e)
        gone = rng.choice(N, 5000, replace=False)
        idx.remove(gone)  # a mutation: the instance quiesces first
        live[gone] = False
        f = batch(q_plain[1])
        check(f)
        extra = R.gen_rows(6, 0, 50_000, DIM)
        idx.add(extra)  # new row count: the workspaces are re-configured
        stored = np.concatenate([stored, R.process_rows(extra, "cosine", "bf16")])
        live = np.concatenate([live, np.ones(len(extra), bool)])
        g = batch(q_plain[2])
        h = batch(q_plain[3])
        check(g)
        check(h)
        ss.finalize_all()
        st = idx.persist_stats()
        assert st["error"] == 0 and st["batches"] - b0 == 7  # a, b, d, e, f, g, h
    finally:
        idx.close()

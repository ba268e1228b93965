"""CPU, world_size 2 over gloo: the row-sharded orchestration (hiprag.dist.ShardedSearch)
-- candidate all-gather, exact merge, guard and collect-mode fallback -- returns the
single-index oracle answer.  Shard search/merge are oracle-backed stand-ins here (host
logic only); the same orchestration drives the HIP kernels and RCCL on the GPU."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

N, DIM, B, K, KC = 3000, 96, 12, 10, 32


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _numpy_merge(cand_all, bound_all, G, Bq, kc, k):
    """Reference semantics of k_merge (exact desc, row asc; guard)."""
    c = cand_all.numpy().reshape(G, Bq, kc, 2)
    rows_all = c.view(np.int64)[..., 1]
    s_out = np.full((Bq, k), -np.inf, np.float32)
    r_out = np.full((Bq, k), -1, np.int64)
    kth = np.full(Bq, -np.inf)
    fail = np.zeros(Bq, np.int32)
    for q in range(Bq):
        sc = c[:, q, :, 0].reshape(-1)
        rw = rows_all[:, q, :].reshape(-1)
        valid = rw >= 0
        sc, rw = sc[valid], rw[valid]
        order = np.lexsort((rw, -sc))
        sc, rw = sc[order], rw[order]
        n = min(k, len(rw))
        s_out[q, :n] = sc[:n]
        r_out[q, :n] = rw[:n]
        maxb = bound_all.numpy()[:, q].max()
        if len(rw) >= k:
            kth[q] = sc[k - 1]
        fail[q] = int(maxb > -np.inf and (len(rw) < k or not kth[q] > maxb))
    return s_out, r_out, kth, fail


def _worker(rank, world, port, result_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import oracle
    from hiprag.dist import ShardedSearch
    from oracle import ref_numpy as R

    lo, hi = N * rank // world, N * (rank + 1) // world
    stored = oracle.c_build_synthetic(5, lo, hi - lo, DIM, "bf16", "cosine", 1)
    rng = np.random.default_rng(0)
    q = rng.standard_normal((B, DIM)).astype(np.float32)
    qn = R.process_queries(q, "cosine")
    e_fake = np.zeros(B)
    e_fake[[1, 7]] = 0.08  # force the guard to fail for two queries -> collect fallback

    class CpuSharded(ShardedSearch):
        def _stream(self):
            return 0

        def _shard_search(self, qt, k, cand, bound, mask_ptr, q_ready=None):
            s, r = oracle.c_search(stored, "bf16", qn[: qt.shape[0]], KC, row_offset=lo, nthreads=1)
            cand.view(torch.int64)[..., 1] = torch.from_numpy(r)
            cand[..., 0] = torch.from_numpy(s)
            full = (hi - lo) > KC
            bound[:] = torch.from_numpy(np.where(full, s[:, -1] + e_fake[: qt.shape[0]], -np.inf))

        def _shard_collect(self, qt, kth, cap, cand, bound, mask_ptr):
            idx = [int(np.nonzero((q == qt[i].numpy()).all(1))[0][0]) for i in range(qt.shape[0])]
            s, r = oracle.c_search(stored, "bf16", qn[idx], cap, row_offset=lo, nthreads=1)
            keep = s >= (kth.numpy()[:, None] - e_fake[idx][:, None])
            s = np.where(keep, s, -np.inf)
            r = np.where(keep, r, -1)
            cand.view(torch.int64)[..., 1] = torch.from_numpy(r)
            cand[..., 0] = torch.from_numpy(s)
            bound[:] = torch.from_numpy(np.where(keep.all(1), np.inf, -np.inf))

        def _merge(self, cand_all, bound_all, G, Bq, kc, k, s_out, r_out, kth, fail):
            s, r, kt, f = _numpy_merge(cand_all, bound_all, G, Bq, kc, k)
            s_out.copy_(torch.from_numpy(s))
            r_out.copy_(torch.from_numpy(r))
            kth.copy_(torch.from_numpy(kt))
            fail.copy_(torch.from_numpy(f))

    ss = CpuSharded(index=None, row_offset=lo, max_batch=B, device=torch.device("cpu"))
    s, r = ss.search(torch.from_numpy(q), K)
    # the same batch known only to rank 1: broadcast first (src_rank), identical results
    q_in = torch.from_numpy(q) if rank == 1 else torch.zeros((B, DIM))
    s2, r2 = ss.search(q_in, K, src_rank=1)
    assert torch.equal(s2, s) and torch.equal(r2, r)
    if rank == 0:
        np.savez(result_path, s=s.numpy(), r=r.numpy())
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_sharded_search_matches_single_index(tmp_path):
    import oracle
    from oracle import ref_numpy as R

    path = str(tmp_path / "res.npz")
    mp.start_processes(_worker, args=(2, _free_port(), path), nprocs=2, join=True, start_method="spawn")
    got = np.load(path)
    stored = oracle.c_build_synthetic(5, 0, N, DIM, "bf16", "cosine", 2)
    q = np.random.default_rng(0).standard_normal((B, DIM)).astype(np.float32)
    s_ref, r_ref = oracle.c_search(stored, "bf16", R.process_queries(q, "cosine"), K)
    np.testing.assert_array_equal(got["r"], r_ref)
    np.testing.assert_array_equal(got["s"], s_ref.astype(np.float32))


def test_merge_guard_semantics():
    """Guard: fail iff some shard still hides rows that might beat the k-th result."""
    cand = torch.zeros((2, 1, 3, 2), dtype=torch.float64)
    cand[0, 0, :, 0] = torch.tensor([0.9, 0.5, 0.4], dtype=torch.float64)
    cand[1, 0, :, 0] = torch.tensor([0.8, 0.7, 0.1], dtype=torch.float64)
    cand.view(torch.int64)[0, 0, :, 1] = torch.tensor([3, 5, 9])
    cand.view(torch.int64)[1, 0, :, 1] = torch.tensor([100, 101, 102])
    s, r, kth, fail = _numpy_merge(cand, torch.tensor([[0.3], [-np.inf]]), 2, 1, 3, 2)
    assert r.tolist() == [[3, 100]] and kth[0] == 0.8 and fail[0] == 0
    s, r, kth, fail = _numpy_merge(cand, torch.tensor([[0.85], [-np.inf]]), 2, 1, 3, 2)
    assert fail[0] == 1

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


class StubRccl:
    """A ctypes-shaped stand-in for librccl.so (the entry points RcclComm binds, same argument conventions) that
    moves the bytes between the ranks with gloo on the host -- so RcclComm's G > 1 control flow (unique-id
    broadcast, ncclCommInitRank(G, uid, rank), rank-ordered all-gather, broadcast, destroy) runs on CPU.  Pointers
    are host addresses here (CPU tensors)."""

    def __init__(self, uid_bytes: bytes):
        import ctypes

        self.ct, self.uid_bytes, self.calls = ctypes, uid_bytes, []

        def get_error_string(rc):
            return b"stub error"

        def get_unique_id(uid_ref):
            ctypes.memmove(ctypes.addressof(uid_ref._obj), self.uid_bytes, 128)
            self.calls.append(("ncclGetUniqueId",))
            return 0

        def comm_init_rank(comm_ref, nranks, uid, rank):
            self.calls.append(("ncclCommInitRank", int(nranks), bytes(uid.internal), int(rank)))
            comm_ref._obj.value = 0x5EED
            return 0

        def all_gather(send, recv, count, dtype, comm, stream):
            n = int(count.value)
            assert dtype == 1 and comm.value == 0x5EED  # uint8, the communicator InitRank returned
            mine = torch.frombuffer(bytearray(ctypes.string_at(send.value, n)), dtype=torch.uint8)
            every = [torch.empty(n, dtype=torch.uint8) for _ in range(dist.get_world_size())]
            dist.all_gather(every, mine)
            for r, t in enumerate(every):  # rank r's bytes at offset r * count (ncclAllGather's layout)
                ctypes.memmove(recv.value + r * n, t.numpy().tobytes(), n)
            self.calls.append(("ncclAllGather", n))
            return 0

        def broadcast(send, recv, count, dtype, root, comm, stream):
            n = int(count.value)
            t = torch.frombuffer(bytearray(ctypes.string_at(send.value, n)), dtype=torch.uint8)
            dist.broadcast(t, int(root))
            ctypes.memmove(recv.value, t.numpy().tobytes(), n)
            self.calls.append(("ncclBroadcast", n, int(root)))
            return 0

        def comm_destroy(comm):
            self.calls.append(("ncclCommDestroy",))
            return 0

        self.ncclGetErrorString = get_error_string
        self.ncclGetUniqueId = get_unique_id
        self.ncclCommInitRank = comm_init_rank
        self.ncclAllGather = all_gather
        self.ncclBroadcast = broadcast
        self.ncclCommDestroy = comm_destroy


def _rccl_worker(rank, world, port, result_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import oracle
    from hiprag.dist import ShardedSearch, _record_len
    from oracle import ref_numpy as R

    lo, hi = N * rank // world, N * (rank + 1) // world
    bounds = [(N * g // world, N * (g + 1) // world) for g in range(world)]
    stored = oracle.c_build_synthetic(5, lo, hi - lo, DIM, "bf16", "cosine", 1)
    q = np.random.default_rng(0).standard_normal((B, DIM)).astype(np.float32)
    qn = R.process_queries(q, "cosine")
    stub = StubRccl(uid_bytes=bytes([rank * 7 + 3]) * 128 if rank == 0 else bytes(128))
    seen = {}

    class CpuRccl(ShardedSearch):
        def _stream(self):
            return 0

        def _shard_search(self, qt, k, cand, bound, mask_ptr, q_ready=None):
            s, r = oracle.c_search(stored, "bf16", qn[: qt.shape[0]], KC, row_offset=lo, nthreads=1)
            cand.view(torch.int64)[..., 1] = torch.from_numpy(r)
            cand[..., 0] = torch.from_numpy(s)
            bound[:] = torch.from_numpy(s[:, -1])

        def _merge(self, cand_all, bound_all, G, Bq, kc, k, s_out, r_out, kth, fail):
            # the packed records as the product's k_merge reads them: rank g's record at g * (record bytes)
            assert cand_all.stride(0) * 8 == _record_len(Bq, kc) * 8 and bound_all.stride(0) == cand_all.stride(0)
            rows = cand_all.contiguous().view(torch.int64)[..., 1].numpy()
            for g, (a, b) in enumerate(bounds):  # rank order: row g of the gather holds rank g's shard rows
                assert ((rows[g] >= a) & (rows[g] < b)).all(), (g, rows[g].min(), rows[g].max())
            seen["merged"] = seen.get("merged", 0) + 1
            s, r, kt, f = _numpy_merge(cand_all, bound_all, G, Bq, kc, k)
            s_out.copy_(torch.from_numpy(s))
            r_out.copy_(torch.from_numpy(r))
            kth.copy_(torch.from_numpy(kt))
            fail.copy_(torch.from_numpy(f))

    ss = CpuRccl(index=None, row_offset=lo, max_batch=B, device=torch.device("cpu"), kc=KC, rccl_lib=stub)
    assert ss.rccl is not None and ss.transport.startswith("rccl") and ss.rccl.G == world
    s, r = ss.search(torch.from_numpy(q), K)
    q_in = torch.from_numpy(q) if rank == 1 else torch.zeros((B, DIM))
    s2, r2 = ss.search(q_in, K, src_rank=1)  # the batch known to rank 1 only: ncclBroadcast from root 1
    assert torch.equal(s2, s) and torch.equal(r2, r)
    ss.close()
    names = [c[0] for c in stub.calls]
    init = [c for c in stub.calls if c[0] == "ncclCommInitRank"][0]
    out = {"rank": rank, "names": names, "init_G": init[1], "init_rank": init[3], "uid": init[2].hex(),
           "merged": seen["merged"], "ag": [c[1] for c in stub.calls if c[0] == "ncclAllGather"],
           "bc": [c[1:] for c in stub.calls if c[0] == "ncclBroadcast"]}
    import json

    with open(f"{result_path}.{rank}.json", "w") as f:
        json.dump(out, f)
    if rank == 0:
        np.savez(result_path, s=s.numpy(), r=r.numpy())
    dist.barrier()
    dist.destroy_process_group()


def test_rccl_comm_two_ranks_with_stub_library(tmp_path):
    """RcclComm's G > 1 control flow on CPU -- the unique id rank 0 draws reaches rank 1 through
    the process-group broadcast, every rank calls ncclCommInitRank(G, that id, its rank), the all-gathered records
    arrive in rank order and the merge reads them with the packed record stride, and the answer is the single-index
    oracle's."""
    import json

    import oracle
    from hiprag.dist import _record_len
    from oracle import ref_numpy as R

    path = str(tmp_path / "rccl")
    mp.start_processes(_rccl_worker, args=(2, _free_port(), path), nprocs=2, join=True, start_method="spawn")
    per = [json.load(open(f"{path}.{r}.json")) for r in range(2)]
    uid0 = (bytes([3]) * 128).hex()
    for r, o in enumerate(per):
        assert o["init_G"] == 2 and o["init_rank"] == r and o["uid"] == uid0  # rank 1 never drew an id itself
        assert o["names"][-1] == "ncclCommDestroy"
        assert o["ag"] == [_record_len(B, KC) * 8] * 2  # one all-gather of the packed record per batch
        assert o["bc"] == [[B * DIM * 4, 1]]            # the src_rank batch: one broadcast from root 1
        assert o["merged"] == 2
    assert "ncclGetUniqueId" in per[0]["names"] and "ncclGetUniqueId" not in per[1]["names"]
    got = np.load(path + ".npz")
    stored = oracle.c_build_synthetic(5, 0, N, DIM, "bf16", "cosine", 2)
    q = np.random.default_rng(0).standard_normal((B, DIM)).astype(np.float32)
    s_ref, r_ref = oracle.c_search(stored, "bf16", R.process_queries(q, "cosine"), K)
    np.testing.assert_array_equal(got["r"], r_ref)
    np.testing.assert_array_equal(got["s"], s_ref.astype(np.float32))


# ---------------------------------------------------------------- ties across the shard boundary, k beyond kc
NT, DUP_LO, DUP_HI = 6000, 2000, 4000  # 2,000 copies of one row straddling the rank boundary at 3,000


def _ties_stored(lo, hi):
    """Stored (bf16, cosine-processed) rows [lo, hi) of the ties corpus: the synthetic rows with rows
    [DUP_LO, DUP_HI) replaced by copies of row 77."""
    import oracle

    x = oracle.c_build_synthetic(5, lo, hi - lo, DIM, "bf16", "cosine", 1)
    dup = oracle.c_build_synthetic(5, 77, 1, DIM, "bf16", "cosine", 1)[0]
    a, b = max(lo, DUP_LO), min(hi, DUP_HI)
    if a < b:
        x[a - lo:b - lo] = dup
    return x


def _ties_queries():
    import oracle
    from oracle import ref_numpy as R

    q = np.random.default_rng(3).standard_normal((B, DIM)).astype(np.float32)
    dup = R.dequantize(oracle.c_build_synthetic(5, 77, 1, DIM, "bf16", "cosine", 1), "bf16")[0]
    q[0] = dup          # its top-k is all ties (2,000 equal scores)
    q[4] = dup + 0.01 * q[4]  # near-ties
    return R.process_queries(q, "cosine")


def _numpy_merge_sorted(cand_all, G, Bq, m, k):
    """Reference semantics of k_merge_sorted: the top-k of the union of the ranks' sorted lists."""
    c = cand_all.numpy().reshape(G, Bq, m, 2)
    rows_all = c.view(np.int64)[..., 1]
    s_out = np.full((Bq, k), -np.inf, np.float32)
    r_out = np.full((Bq, k), -1, np.int64)
    for q in range(Bq):
        sc, rw = c[:, q, :, 0].reshape(-1), rows_all[:, q, :].reshape(-1)
        sc, rw = sc[rw >= 0], rw[rw >= 0]
        order = np.lexsort((rw, -sc))[:k]
        s_out[q, :len(order)], r_out[q, :len(order)] = sc[order], rw[order]
    return s_out, r_out


def _ties_worker(rank, world, port, result_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import oracle
    from hiprag.dist import ShardedSearch

    lo, hi = NT * rank // world, NT * (rank + 1) // world
    stored = _ties_stored(lo, hi)
    qn = _ties_queries()
    stub = StubRccl(uid_bytes=bytes([9]) * 128 if rank == 0 else bytes(128))
    seen = {"scan_kc": [], "collect": 0, "exact_m": []}

    def qidx(qt):
        return [int(np.nonzero((qn == qt[i].numpy()).all(1))[0][0]) for i in range(qt.shape[0])]

    class CpuTies(ShardedSearch):
        """Shard pieces with the kernels' contracts: the scan's bound is the k-th candidate's score (ties at
        the boundary fail the guard), a collect window larger than its buffer returns the shard's exact top
        rows (bound -inf), the exhaustive pass returns the sorted exact top-m."""

        def _stream(self):
            return 0

        def _shard_search(self, qt, k, cand, bound, mask_ptr, q_ready=None, kc=None):
            kc = kc or self.kc
            seen["scan_kc"].append(kc)
            s, r = oracle.c_search(stored, "bf16", qn[qidx(qt)], kc, row_offset=lo, nthreads=1)
            cand.view(torch.int64)[..., 1] = torch.from_numpy(r)
            cand[..., 0] = torch.from_numpy(s)
            bound[:] = torch.from_numpy(np.where(r[:, -1] >= 0, s[:, -1], -np.inf))

        def _shard_collect(self, qt, kth, cap, cand, bound, mask_ptr):
            seen["collect"] += 1
            s, r = oracle.c_search(stored, "bf16", qn[qidx(qt)], cap, row_offset=lo, nthreads=1)
            keep = s >= kth.numpy()[:, None]
            full = keep[:, -1]  # the window reaches past the buffer: the shard's exact top-cap instead
            keep |= full[:, None]
            cand.view(torch.int64)[..., 1] = torch.from_numpy(np.where(keep, r, -1))
            cand[..., 0] = torch.from_numpy(np.where(keep, s, -np.inf))
            bound[:] = -np.inf

        def _shard_exact(self, qt, m, cand, mask_ptr):
            seen["exact_m"].append(m)
            s, r = oracle.c_search(stored, "bf16", qn[qidx(qt)], m, row_offset=lo, nthreads=1)
            cand.view(torch.int64)[..., 1] = torch.from_numpy(r)
            cand[..., 0] = torch.from_numpy(s)

        def _merge(self, cand_all, bound_all, G, Bq, kc, k, s_out, r_out, kth, fail):
            s, r, kt, f = _numpy_merge(cand_all, bound_all, G, Bq, kc, k)
            s_out.copy_(torch.from_numpy(s))
            r_out.copy_(torch.from_numpy(r))
            kth.copy_(torch.from_numpy(kt))
            fail.copy_(torch.from_numpy(f))

        def _merge_sorted(self, cand_all, G, Bq, m, k, s_out, r_out):
            s, r = _numpy_merge_sorted(cand_all.contiguous(), G, Bq, m, k)
            s_out.copy_(torch.from_numpy(s))
            r_out.copy_(torch.from_numpy(r))

    ss = CpuTies(index=None, row_offset=lo, max_batch=B, device=torch.device("cpu"), max_k=16, rccl_lib=stub)
    assert ss.kc == 32 and ss.rccl is not None
    out = {}
    for k in (10, 100, 200):
        s, r = ss.search(torch.from_numpy(qn), k)
        out[f"s{k}"], out[f"r{k}"] = s.numpy(), r.numpy()
    s_b, r_b = ss.search(torch.from_numpy(qn) if rank == 1 else torch.zeros((B, DIM)), 200, src_rank=1)
    assert torch.equal(r_b, torch.from_numpy(out["r200"]))
    ss.close()
    out["fallback"], out["exact"] = ss.fallback_queries, ss.exact_queries
    out["scan_kc"], out["collect"], out["exact_m"] = np.array(seen["scan_kc"]), seen["collect"], np.array(seen["exact_m"])
    if rank == 0:
        np.savez(result_path, **out)
    dist.barrier()
    dist.destroy_process_group()


def test_sharded_ties_and_large_k_match_oracle(tmp_path):
    """2,000 duplicate rows straddling the shard boundary and k in {10, 100, 200} -- k above
    the pipelined kc (32) and above HR_MAX_K -- through the stub-RCCL exchange, identical to the single-index
    oracle (ids and score bits); nothing raises."""
    import oracle

    path = str(tmp_path / "ties.npz")
    mp.start_processes(_ties_worker, args=(2, _free_port(), path), nprocs=2, join=True, start_method="spawn")
    got = np.load(path)
    stored = _ties_stored(0, NT)
    qn = _ties_queries()
    for k in (10, 100, 200):
        s_ref, r_ref = oracle.c_search(stored, "bf16", qn, k)
        np.testing.assert_array_equal(got[f"r{k}"], r_ref, err_msg=f"k={k}")
        np.testing.assert_array_equal(got[f"s{k}"], s_ref.astype(np.float32), err_msg=f"k={k}")
    # (row 77 itself ties with its 2,000 copies and comes first)
    assert list(got["r10"][0]) == [77] + list(range(DUP_LO, DUP_LO + 9))
    assert list(got["r200"][0]) == [77] + list(range(DUP_LO, DUP_LO + 199))
    # k = 10: the pipelined scan (kc 32), ties -> collect fallback; k = 100: the scan at kc_for_k(100) = 160, its
    # fallback; k = 200 > HR_MAX_K: the exhaustive pass (twice: the plain and the broadcast batch)
    assert list(got["scan_kc"]) == [32, 160] and int(got["collect"]) >= 2 and int(got["fallback"]) >= 2
    assert list(got["exact_m"]) == [200, 200] and int(got["exact"]) == 2 * B

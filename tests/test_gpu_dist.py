"""GPU: the row-sharded path with the REAL kernels -- 2 ranks (gloo for the tiny candidate
exchange; RCCL needs one GPU per rank) sharing the box's GPU, each holding half the corpus --
returns exactly the single-index answer, including a query that needs the exact fallback."""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

N, DIM, B, K = 40000, 256, 24, 10


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _queries():
    from hiprag import synth

    q, _ = synth.planted_queries(9, N, DIM, B, qseed=4)
    q[5] = synth.corpus_rows(9, [77], DIM)[0]  # its duplicates (planted below) force the fallback
    return q


def _corpus_rows(lo, hi):
    from hiprag import synth

    x = synth.corpus_rows(9, np.arange(lo, hi), DIM)
    dup_rows = np.arange(1000, 40000, 900)  # 44 copies of row 77 spread over both shards (> kc = 32)
    for r in dup_rows[(dup_rows >= lo) & (dup_rows < hi)]:
        x[r - lo] = synth.corpus_rows(9, [77], DIM)[0]
    return x


def _worker(rank, world, port, path):
    import torch
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from hiprag import _native
    from hiprag.dist import ShardedSearch

    torch.cuda.set_device(0)
    lo, hi = N * rank // world, N * (rank + 1) // world
    idx = _native.NativeIndex(DIM, "bf16", "cosine", device=0)
    idx.add(_corpus_rows(lo, hi))
    ss = ShardedSearch(idx, lo, max_batch=B, device=torch.device("cuda", 0))
    q = torch.from_numpy(_queries()).cuda()
    s, r = ss.search(q, K)
    s2 = torch.empty_like(s)
    r2 = torch.empty_like(r)
    ss.finalize(ss.submit(q, K, s_out=s2, r_out=r2))  # pipelined entry points agree
    assert torch.equal(r, r2) and torch.equal(s, s2)
    # the batch known to rank 0 only, broadcast before the scan (early SAMPLE waits for the broadcast)
    ready = torch.cuda.Event()
    ready.record()
    q_in = q if rank == 0 else torch.zeros_like(q)
    s3, r3 = torch.empty_like(s), torch.empty_like(r)
    ss.finalize(ss.submit(q_in, K, s_out=s3, r_out=r3, q_ready=ready, src_rank=0))
    assert torch.equal(r, r3) and torch.equal(s, s3)
    np.savez(f"{path}.{rank}.npz", s=s.cpu().numpy(), r=r.cpu().numpy())
    dist.barrier()
    dist.destroy_process_group()


def test_two_ranks_on_one_gpu_match_single_index(tmp_path):
    import torch.multiprocessing as mp

    from hiprag import _native

    path = str(tmp_path / "res")
    mp.start_processes(_worker, args=(2, _free_port(), path), nprocs=2, join=True, start_method="spawn")
    full = _native.NativeIndex(DIM, "bf16", "cosine")
    full.add(_corpus_rows(0, N))
    s_ref, r_ref = full.search(_queries(), K)
    for rank in range(2):
        got = np.load(f"{path}.{rank}.npz")
        np.testing.assert_array_equal(got["r"], r_ref)
        np.testing.assert_array_equal(got["s"], s_ref)
    assert (r_ref[5] >= 0).all() and len(set(r_ref[5].tolist())) == K


# ---------------------------------------------------------------- early SAMPLE + dual FILTER streams
NE, DIME, BE, KE, NB = 2_200_000, 64, 64, 10, 5  # 1.1M-row shards: large enough for the early mode


def _worker_early(rank, world, port, path):
    import torch
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from hiprag import _native, synth
    from hiprag.dist import ShardedSearch

    torch.cuda.set_device(0)
    lo, hi = NE * rank // world, NE * (rank + 1) // world
    idx = _native.NativeIndex(DIME, "bf16", "cosine", device=0)
    idx.reserve(hi - lo)
    idx.add_synthetic(31, lo, hi - lo)  # the counter-based generator: global rows, any sharding
    ss = ShardedSearch(idx, lo, max_batch=BE, device=torch.device("cuda", 0))
    qs = torch.from_numpy(np.stack([synth.planted_queries(31, NE, DIME, BE, qseed=50 + i)[0] for i in range(NB)])).cuda()
    q_ready = torch.cuda.Event()
    q_ready.record()
    s = torch.empty((NB, BE, KE), dtype=torch.float32, device="cuda")
    r = torch.empty((NB, BE, KE), dtype=torch.int64, device="cuda")
    for i in range(NB):  # pipelined: batch i+1's prep + SAMPLE beside batch i's FILTER, alternating workspaces
        ss.submit(qs[i], KE, s_out=s[i], r_out=r[i], q_ready=q_ready)
    ss.finalize_all()
    torch.cuda.synchronize()
    np.savez(f"{path}.{rank}.npz", s=s.cpu().numpy(), r=r.cpu().numpy())
    dist.barrier()
    dist.destroy_process_group()


def test_two_ranks_early_sample_pipelined_match_oracle(tmp_path):
    """2 ranks x 1.1M-row shards with queries ready by event: the per-shard early SAMPLE on the pre
    stream and the dual FILTER streams, then the exchange + merge; every batch identical to the
    CPU oracle over the whole corpus."""
    import torch.multiprocessing as mp

    import oracle
    from hiprag import synth
    from oracle import ref_numpy as R

    path = str(tmp_path / "res")
    mp.start_processes(_worker_early, args=(2, _free_port(), path), nprocs=2, join=True, start_method="spawn")
    stored = oracle.c_build_synthetic(31, 0, NE, DIME, "bf16", "cosine")
    got = [np.load(f"{path}.{rank}.npz") for rank in range(2)]
    for i in range(NB):
        q, _ = synth.planted_queries(31, NE, DIME, BE, qseed=50 + i)
        s_ref, r_ref = oracle.c_search(stored, "bf16", R.process_queries(q, "cosine"), KE)
        for g in got:
            np.testing.assert_array_equal(g["r"][i], r_ref)
            np.testing.assert_array_equal(g["s"][i], s_ref.astype(np.float32))


# ---------------------------------------------------------------- ties across the boundary, k beyond kc
NT, DIMT, BT = 200_000, 256, 16
DUP_LO, DUP_HI = 99_000, 101_000  # 2,000 copies of row 77 straddling the rank boundary at 100,000
KS = (10, 100, 200)


def _ties_rows(lo, hi):
    from hiprag import synth

    x = synth.corpus_rows(13, np.arange(lo, hi), DIMT)
    a, b = max(lo, DUP_LO), min(hi, DUP_HI)
    if a < b:
        x[a - lo:b - lo] = synth.corpus_rows(13, [77], DIMT)[0]
    return x


def _ties_queries():
    from hiprag import synth

    q = np.random.default_rng(17).standard_normal((BT, DIMT)).astype(np.float32)
    dup = synth.corpus_rows(13, [77], DIMT)[0]
    q[0] = dup
    q[3] = dup + 0.02 * q[3]
    return q


def _worker_ties(rank, world, port, path):
    import torch
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from hiprag import _native
    from hiprag.dist import ShardedSearch

    torch.cuda.set_device(0)
    lo, hi = NT * rank // world, NT * (rank + 1) // world
    idx = _native.NativeIndex(DIMT, "bf16", "cosine", device=0)
    idx.add(_ties_rows(lo, hi))
    ss = ShardedSearch(idx, lo, max_batch=BT, device=torch.device("cuda", 0), max_k=16)
    q = torch.from_numpy(_ties_queries()).cuda()
    out = {}
    for k in KS:
        s, r = ss.search(q, k)
        out[f"s{k}"], out[f"r{k}"] = s.cpu().numpy(), r.cpu().numpy()
    out["fallback"], out["exact"] = ss.fallback_queries, ss.exact_queries
    ss.close()
    np.savez(f"{path}.{rank}.npz", **out)
    dist.barrier()
    dist.destroy_process_group()


def test_two_ranks_ties_and_large_k_match_oracle(tmp_path):
    """VERDICT r05 next #1 on the real kernels: 2 ranks, 2,000 duplicate rows across the boundary, k = 10 (pipelined
    kc 32, ties -> collect windows larger than their buffer -> per-shard exhaustive), k = 100 (the scan at kc 160)
    and k = 200 > HR_MAX_K (hr_index_search_shard_exact + hr_merge_sorted): ids and score bits equal the oracle."""
    import torch.multiprocessing as mp

    import oracle
    from oracle import ref_numpy as R

    path = str(tmp_path / "ties")
    mp.start_processes(_worker_ties, args=(2, _free_port(), path), nprocs=2, join=True, start_method="spawn")
    stored = R.process_rows(_ties_rows(0, NT), "cosine", "bf16")
    qn = R.process_queries(_ties_queries(), "cosine")
    for rank in range(2):
        got = np.load(f"{path}.{rank}.npz")
        for k in KS:
            s_ref, r_ref = oracle.c_search(stored, "bf16", qn, k)
            np.testing.assert_array_equal(got[f"r{k}"], r_ref, err_msg=f"rank {rank} k={k}")
            np.testing.assert_array_equal(got[f"s{k}"], s_ref.astype(np.float32), err_msg=f"rank {rank} k={k}")
        assert int(got["fallback"]) >= 1 and int(got["exact"]) == BT
        assert list(got["r200"][0][:3]) == [77, DUP_LO, DUP_LO + 1]


def test_shard_exact_and_merge_sorted_vs_oracle():
    """hr_index_search_shard_exact (row offset, mask, m past the shard's rows) and hr_merge_sorted over 3 shards."""
    import torch

    import oracle
    from hiprag import _native, synth
    from oracle import ref_numpy as R

    n, d, b, m = 30_000, 128, 8, 300
    x = synth.corpus_rows(21, np.arange(n), d)
    x[5000:5600] = x[11]  # ties inside and across shards
    x[10000:10500] = x[11]
    q = np.random.default_rng(5).standard_normal((b, d)).astype(np.float32)
    q[0] = x[11]
    allowed = np.ones(n, bool)
    allowed[::7] = False
    bounds = [(0, 10000), (10000, 29900), (29900, n)]  # the last shard holds 100 rows < m
    qd = torch.from_numpy(q).cuda()
    recs = torch.empty((3, b, m, 2), dtype=torch.float64, device="cuda")
    for g, (lo, hi) in enumerate(bounds):
        idx = _native.NativeIndex(d, "bf16", "cosine", device=0)
        idx.add(x[lo:hi])
        mask = torch.from_numpy(oracle.mask_from_bool(allowed[lo:hi]).view(np.int64)).cuda()
        idx.search_shard_exact(qd.data_ptr(), b, m, lo, recs[g].data_ptr(), mask_ptr=mask.data_ptr())
        torch.cuda.synchronize()
        stored = R.process_rows(x[lo:hi], "cosine", "bf16")
        s_ref, r_ref = oracle.c_search(stored, "bf16", R.process_queries(q, "cosine"), m,
                                       oracle.mask_from_bool(allowed[lo:hi]), row_offset=lo)
        got = recs[g].cpu().numpy()
        np.testing.assert_array_equal(got[..., 1].view(np.int64), r_ref, err_msg=f"shard {g}")
        np.testing.assert_array_equal(got[..., 0], s_ref, err_msg=f"shard {g}")
        idx.close()
    all_rec = recs.cpu().numpy()
    sc_all = all_rec[..., 0].transpose(1, 0, 2).reshape(b, -1)
    rw_all = all_rec[..., 1].view(np.int64).transpose(1, 0, 2).reshape(b, -1)
    s_glob, r_glob = oracle.c_search(R.process_rows(x, "cosine", "bf16"), "bf16", R.process_queries(q, "cosine"), m,
                                     oracle.mask_from_bool(allowed))
    for k in (10, 250, 700, 1000):  # 1000 > the 3 * 300 - padding records there are
        s = torch.empty((b, k), dtype=torch.float32, device="cuda")
        r = torch.empty((b, k), dtype=torch.int64, device="cuda")
        _native.merge_sorted(0, recs.data_ptr(), 3, b, m, k, s.data_ptr(), r.data_ptr())
        torch.cuda.synchronize()
        for qi in range(b):  # the top-k of the union of the lists (score desc, row asc), padded
            ok = rw_all[qi] >= 0
            order = np.lexsort((rw_all[qi][ok], -sc_all[qi][ok]))[:k]
            want_r = np.full(k, -1, np.int64)
            want_s = np.full(k, -np.inf, np.float32)
            want_r[:len(order)] = rw_all[qi][ok][order]
            want_s[:len(order)] = sc_all[qi][ok][order]
            np.testing.assert_array_equal(r.cpu().numpy()[qi], want_r, err_msg=f"k={k} q={qi}")
            np.testing.assert_array_equal(s.cpu().numpy()[qi], want_s, err_msg=f"k={k} q={qi}")
        kk = min(k, m)  # within m every shard contributed its whole top: the global order
        np.testing.assert_array_equal(r.cpu().numpy()[:, :kk], r_glob[:, :kk], err_msg=f"k={k}")
        np.testing.assert_array_equal(s.cpu().numpy()[:, :kk], s_glob[:, :kk].astype(np.float32), err_msg=f"k={k}")

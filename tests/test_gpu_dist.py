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

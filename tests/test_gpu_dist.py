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

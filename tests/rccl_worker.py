"""Child process of tests/test_gpu_rccl.py: the production exchange of hiprag.dist.ShardedSearch
through a REAL RCCL process group (backend "nccl", world size 1, one GPU).

Usage: python tests/rccl_worker.py <port> <queries.npz> <out.npz> <rows> <dim>
       python tests/rccl_worker.py ties <port> <rows.npz> <out.npz>   (duplicate rows, k = 10 / 100 / 200)

At world size 1 the exchange is normally a local copy; ``force_collective=True`` sends the packed
per-shard records through ``all_gather_into_tensor`` and src_rank batches through ``broadcast`` on the
tail / scan streams -- the branch an 8-GPU node runs (dist.py ``_all_gather`` / ``_broadcast``).  A
subclass forces every query of one batch through the collect fallback, so ``_fallback``'s second
all-gather runs too.  Every exchange is counted (ShardedSearch.collective_calls) and the backend and transport
(RCCL called directly on the tail / scan streams, dist.RcclComm) are reported, so the parent can assert the RCCL
branch executed.  Runs in its own process so a hung communicator is bounded by the
parent's timeout.
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for _p in (REPO, os.path.join(REPO, "youtu-rag_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402


def main(port: int, q_path: str, out_path: str, rows: int, dim: int) -> None:
    import torch
    import torch.distributed as dist

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    # the process group first, with its device: RCCL's communicator is created eagerly on it
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1, device_id=dev)
    backend = dist.get_backend()

    from hiprag import _native
    from hiprag.dist import ShardedSearch

    q = np.load(q_path)["q"]  # (2, B, dim): planted batch, isotropic batch
    nb, B, _ = q.shape
    k = 10
    idx = _native.NativeIndex(dim, "bf16", "cosine", device=0)
    idx.reserve(rows)
    idx.add_synthetic(0, 0, rows)
    qd = torch.from_numpy(q).to(dev)
    ready = torch.cuda.Event()
    ready.record()

    ss = ShardedSearch(idx, 0, max_batch=B, device=dev, max_k=k, force_collective=True)
    n_out = 6
    s = torch.empty((n_out, B, k), dtype=torch.float32, device=dev)
    r = torch.empty((n_out, B, k), dtype=torch.int64, device=dev)
    # 0-3: the bench's pipelined path (scan + tail streams, early SAMPLE, two slots), planted / isotropic
    for i in range(4):
        ss.submit(qd[i % 2], k, s_out=s[i], r_out=r[i], q_ready=ready)
    ss.finalize_all()
    # 4: a batch known to rank 0 only, broadcast on the scan stream before the scan
    ss.finalize(ss.submit(qd[0].clone(), k, s_out=s[4], r_out=r[4], q_ready=ready, src_rank=0))

    # 5: every query of the isotropic batch forced through the collect fallback (second all-gather)
    class ForcedFallback(ShardedSearch):
        def _failed_queries(self, slot, B):
            return np.arange(B)

    ff = ForcedFallback(idx, 0, max_batch=B, device=dev, max_k=k, force_collective=True)
    ff.search(qd[1], k, s_out=s[5], r_out=r[5])
    torch.cuda.synchronize()
    calls = {c: ss.collective_calls[c] + ff.collective_calls[c] for c in ("all_gather", "broadcast")}
    np.savez(out_path, s=s.cpu().numpy(), r=r.cpu().numpy(), backend=np.array(backend),
             ag=np.array(calls["all_gather"]), bc=np.array(calls["broadcast"]), transport=np.array(ss.transport),
             persist=np.array(idx.persist_stats()["batches"]))
    ss.close()
    ff.close()
    dist.destroy_process_group()


def main_ties(port: int, in_path: str, out_path: str) -> None:
    """The exact paths through real RCCL: a corpus with 2,000 copies of one row and k = 10 (pipelined kc 32; the
    ties fail the guard and overflow the collect window -> the shard's exhaustive top rows), k = 100 (the scan at
    kc_for_k(100) = 160) and k = 200 > HR_MAX_K (hr_index_search_shard_exact, all-gather, hr_merge_sorted)."""
    import torch
    import torch.distributed as dist

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1, device_id=dev)
    from hiprag import _native
    from hiprag.dist import ShardedSearch

    z = np.load(in_path)
    x, q = z["x"], z["q"]
    idx = _native.NativeIndex(x.shape[1], "bf16", "cosine", device=0)
    idx.add(x)
    ss = ShardedSearch(idx, 0, max_batch=q.shape[0], device=dev, max_k=16, force_collective=True)
    qd = torch.from_numpy(q).to(dev)
    out = {}
    for k in (10, 100, 200):
        s, r = ss.search(qd, k)
        out[f"s{k}"], out[f"r{k}"] = s.cpu().numpy(), r.cpu().numpy()
    torch.cuda.synchronize()
    out.update(ag=np.array(ss.collective_calls["all_gather"]), transport=np.array(ss.transport),
               fallback=np.array(ss.fallback_queries), exact=np.array(ss.exact_queries))
    np.savez(out_path, **out)
    ss.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    if sys.argv[1] == "ties":
        main_ties(int(sys.argv[2]), sys.argv[3], sys.argv[4])
    else:
        main(int(sys.argv[1]), sys.argv[2], sys.argv[3], int(sys.argv[4]), int(sys.argv[5]))

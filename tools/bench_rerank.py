#!/usr/bin/env python3
"""BASELINE.json configs[4] on one MI355X: "Hybrid rerank: 50M×1024 fp16 ANN candidate-gen +
cross-encoder rerank top-100, 8 MI355X" -- measured as ONE rank of the 8-GPU job.

Per rank: a 50M/8 = 6.25M-row shard of a clustered synthetic fp16 corpus (1024-d), an IVF-flat
index over it (shared-centroid lists, hiprag.ivf) and, for the recall check, the exact
brute-force index over the same rows.  Per batch of B queries:
  stage 1  IVF top-100 candidates of the shard (hr_ivf_search: exact within the probed lists);
           on 8 ranks the per-shard top-100s are merged by one all-gather (dist.py), so stage 1
           per rank is what is timed here;
  stage 2  cross-encoder rerank of each query's 100 candidates to the top 10 (TorchRocmReranker,
           bge-reranker-base shape, random init, bf16).  On 8 ranks each rank reranks B/8 of the
           batch's queries, so the per-rank stage-2 work is B/8 queries x 100 pairs; this tool
           times stage 2 for --rerank-queries queries (default B/8) and reports both.
Node-level QPS = B / max(stage-1 time, stage-2 time of B/8 queries) if the two stages of
consecutive batches overlap, and B / (sum) if they do not; both are printed.

Usage: python tools/bench_rerank.py [--rows 6250000 --nlist 8192 --nprobe 32 --batch 64 --steps 10]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "youtu-rag_amd"), REPO]


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--rows", type=int, default=6_250_000)
    p.add_argument("--dim", type=int, default=1024)
    p.add_argument("--dtype", default="f16")
    p.add_argument("--nlist", type=int, default=8192)
    p.add_argument("--nprobe", type=int, default=32)
    p.add_argument("--centers", type=int, default=20000)
    p.add_argument("--spread", type=float, default=0.7)
    p.add_argument("--batch", type=int, default=64)
    p.add_argument("--k", type=int, default=100)
    p.add_argument("--final-k", type=int, default=10)
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--rerank-queries", type=int, default=0, help="queries reranked per step (default batch/8)")
    p.add_argument("--rerank-batch", type=int, default=512)
    p.add_argument("--passage-words", type=int, default=110)
    p.add_argument("--no-exact", action="store_true")
    args = p.parse_args()

    import numpy as np
    import torch

    from hiprag import _native
    from hiprag.ivf import IvfIndex
    from hiprag.rag import Chunk, RetrievalResult
    from hiprag.rag.rerankers import TorchRocmReranker

    dev = torch.device("cuda", 0)
    N, D = args.rows, args.dim
    st = lambda: torch.cuda.current_stream(dev).cuda_stream  # noqa: E731

    # clustered synthetic corpus: row r = unit(center[c(r)]) + spread * unit(noise_r), generated on the GPU
    centers = torch.empty((args.centers, D), dtype=torch.float32, device=dev)
    _native.gen_rows_device(7, 0, args.centers, D, centers.data_ptr(), st())
    centers = torch.nn.functional.normalize(centers, dim=1)

    def rows(i0, i1):
        noise = torch.empty((i1 - i0, D), dtype=torch.float32, device=dev)
        _native.gen_rows_device(11, i0, i1 - i0, D, noise.data_ptr(), st())
        c = (torch.arange(i0, i1, device=dev, dtype=torch.int64) * 2654435761) % args.centers
        return centers[c] + args.spread * torch.nn.functional.normalize(noise, dim=1)

    t0 = time.time()
    ivf = IvfIndex(D, args.nlist, dtype=args.dtype, metric="cosine")
    sample = rows(0, min(N, args.nlist * 32))
    ivf.train(sample, iters=10, seed=0)
    del sample
    torch.cuda.synchronize()
    log(f"trained {args.nlist} lists in {time.time() - t0:.1f}s")
    t0 = time.time()
    ivf.build(N, rows)
    torch.cuda.synchronize()
    sizes = (ivf.list_tiles[1:] - ivf.list_tiles[:-1]).float() * 32
    log(f"built IVF lists over {N} rows in {time.time() - t0:.1f}s (max list {int(sizes.max())} rows, "
        f"{ivf.list_tiles[-1].item() * 32 / N:.3f}x padded)")
    flat = None
    if not args.no_exact:
        t0 = time.time()
        flat = _native.NativeIndex(D, args.dtype, "cosine")
        flat.reserve(N)
        for i in range(0, N, 1 << 18):
            x = rows(i, min(N, i + (1 << 18))).contiguous()
            flat.add_device(x.data_ptr(), x.shape[0], st())
        torch.cuda.synchronize()
        log(f"built exact index in {time.time() - t0:.1f}s")

    B, K = args.batch, args.k
    nb = args.warmup + args.steps
    g = torch.Generator(device=dev)
    g.manual_seed(5)
    qs = []
    for i in range(nb):
        j = torch.randint(0, N, (B,), generator=g, device=dev)
        base = torch.cat([rows(int(r), int(r) + 1) for r in j.tolist()])
        qs.append((base + 0.1 * torch.randn(base.shape, generator=g, device=dev)).contiguous())
    cand = torch.empty((nb, B, K, 2), dtype=torch.float64, device=dev)
    bound = torch.empty((nb, B), dtype=torch.float64, device=dev)

    # stage 1: IVF candidates
    for i in range(args.warmup):
        ivf.search_candidates(qs[i], K, args.nprobe, cand[i], bound[i])
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for i in range(args.warmup, nb):
        ivf.search_candidates(qs[i], K, args.nprobe, cand[i], bound[i])
    e1.record()
    torch.cuda.synchronize()
    ivf_ms = e0.elapsed_time(e1) / args.steps
    ids = cand.view(torch.int64)[..., 1]
    # bytes the list scan reads per batch: every tile of every (query, probed list)
    probes = torch.empty((B, args.nprobe, 2), dtype=torch.float64, device=dev)
    ivf.search_candidates(qs[args.warmup], K, args.nprobe, cand[args.warmup], bound[args.warmup], probes=probes)
    pl = probes.view(torch.int64)[..., 1]
    tiles = int((ivf.list_tiles[pl + 1] - ivf.list_tiles[pl]).sum().item())
    scan_bytes = tiles * 32 * D * 2
    ivf_gbs = scan_bytes / (ivf_ms * 1e-3) / 1e9

    out = {"config": "configs[4] per rank: 6.25M x 1024 fp16 shard (50M / 8), IVF-flat top-100, "
                     "cross-encoder rerank to top-10",
           "rows": N, "dim": D, "dtype": args.dtype, "nlist": args.nlist, "nprobe": args.nprobe, "batch": B,
           "stage1_ivf_ms_per_batch": round(ivf_ms, 4), "stage1_ivf_qps_per_rank": round(B / ivf_ms * 1e3, 1),
           "stage1_scan_bytes_per_batch": scan_bytes, "stage1_scan_bytes_over_batch_time_GBps": round(ivf_gbs, 1)}

    if flat is not None:  # recall of the IVF candidates against the exact search, and the exact search's cost
        ex_s = torch.empty((B, K), dtype=torch.float32, device=dev)
        ex_r = torch.empty((B, K), dtype=torch.int64, device=dev)
        flat.search_device(qs[args.warmup].data_ptr(), B, K, ex_s.data_ptr(), ex_r.data_ptr(), stream=st())
        torch.cuda.synchronize()
        got = ids[args.warmup].cpu().numpy()
        ref = ex_r.cpu().numpy()
        out["stage1_recall_at_100"] = round(float(np.mean([len(set(got[b]) & set(ref[b])) / K for b in range(B)])), 4)
        out["stage1_recall_at_10"] = round(float(np.mean([len(set(got[b][:10]) & set(ref[b][:10])) / 10
                                                          for b in range(B)])), 4)
        t1 = time.perf_counter()
        for i in range(args.warmup, nb):
            flat.search_device(qs[i].data_ptr(), B, K, ex_s.data_ptr(), ex_r.data_ptr(), stream=st())
        torch.cuda.synchronize()
        out["exact_bruteforce_ms_per_batch"] = round((time.perf_counter() - t1) * 1e3 / args.steps, 4)

    # stage 2: cross-encoder rerank of each query's 100 candidates
    rq = args.rerank_queries or max(1, B // 8)
    rr = TorchRocmReranker(preset="bge-reranker-base", dtype="bfloat16", batch_size=args.rerank_batch,
                           max_length=512)
    vocab = [f"tok{i}" for i in range(20000)]
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from flops import EncoderFlops, mfma_block

    counter = EncoderFlops(rr.model, getattr(rr, "unpadded", None))

    def passage(row: int) -> str:  # stored chunk text of a row (deterministic synthetic words)
        r = np.random.default_rng(row)
        return " ".join(r.choice(vocab, args.passage_words))

    def results_of(i, b):
        return [RetrievalResult(chunk=Chunk(id=str(int(x)), document_id="d", content=texts[int(x)], chunk_index=0),
                                score=float(s), rank=n + 1)
                for n, (s, x) in enumerate(zip(cand[i, b, :, 0].tolist(), ids[i, b].tolist())) if x >= 0]

    texts = {int(x): passage(int(x)) for i in range(nb) for b in range(rq) for x in ids[i, b].tolist() if x >= 0}
    queries = [" ".join(np.random.default_rng(10_000 + i).choice(vocab, 12)) for i in range(nb * rq)]
    work = [([queries[i * rq + b] for b in range(rq)], [results_of(i, b) for b in range(rq)]) for i in range(nb)]
    # cold pass over the warmup batches tokenises their passages; the timed batches are cold too
    t_tok = time.perf_counter()
    for i in range(args.warmup):
        rr.rerank_batch(*work[i], top_k=args.final_k)
    torch.cuda.synchronize()
    log(f"rerank warmup {time.perf_counter() - t_tok:.2f}s")
    # passage token ids come from the ingest-time cache (TorchRocmReranker.warm), as the chunk text is
    # tokenised there anyway; the cold tokenisation cost is reported separately
    t_tok = time.perf_counter()
    for i in range(args.warmup, nb):
        rr.warm([r.chunk.content for rs in work[i][1] for r in rs])
    tok_ms = (time.perf_counter() - t_tok) * 1e3 / args.steps
    counter.reset()
    t1 = time.perf_counter()
    pairs = 0
    for i in range(args.warmup, nb):
        res = rr.rerank_batch(*work[i], top_k=args.final_k)
        pairs += sum(len(r) for r in work[i][1])
    torch.cuda.synchronize()
    rr_ms = (time.perf_counter() - t1) * 1e3 / args.steps
    out["stage2_mfma"] = mfma_block(counter.totals(), rr_ms * args.steps / 1e3,
                                    what="cross-encoder forward of the timed steps (tools/flops.py)")
    assert all(len(r) == args.final_k for r in res)
    out.update({"stage2_passage_tokenise_ms_per_step_cold": round(tok_ms, 2),
                "stage2_rerank_queries_per_step": rq, "stage2_pairs_per_step": pairs // args.steps,
                "stage2_ms_per_step": round(rr_ms, 3), "stage2_pairs_per_s": round(pairs / args.steps / rr_ms * 1e3, 1),
                "stage2_rerank_qps_per_rank": round(rq / rr_ms * 1e3, 2)})
    # node (8 ranks): each batch of B queries -> stage 1 on every rank + stage 2 of B/8 queries per rank
    per_batch_serial = ivf_ms + rr_ms * (B / 8) / rq
    per_batch_overlap = max(ivf_ms, rr_ms * (B / 8) / rq)
    out["node8_qps_serial"] = round(B / per_batch_serial * 1e3, 1)
    out["node8_qps_overlapped"] = round(B / per_batch_overlap * 1e3, 1)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()

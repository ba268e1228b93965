#!/usr/bin/env python3
"""IVF-flat candidate generation vs the exact scan on one 6.25M x 1024 f16 shard (BASELINE configs[4]
per rank), on a clustered and an isotropic corpus.  Per distribution: IVF ms/batch (B=64, top-100),
the probed bytes per batch and their rate, recall@100/@10 against the exact search of the same rows,
and the exact search's ms/batch.  One JSON line per distribution.
Usage: python tools/bench_ivf.py [--rows 6250000 --nlist 8192 --nprobe 32 --steps 10 --dist clustered,isotropic]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "youtu-rag_amd"), REPO]


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--rows", type=int, default=6_250_000)
    p.add_argument("--dim", type=int, default=1024)
    p.add_argument("--dtype", default="f16")
    p.add_argument("--nlist", type=int, default=8192)
    p.add_argument("--nprobe", type=int, default=32)
    p.add_argument("--batch", type=int, default=64)
    p.add_argument("--k", type=int, default=100)
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--dist", default="clustered,isotropic")
    p.add_argument("--centers", type=int, default=20000)
    p.add_argument("--spread", type=float, default=0.7)
    args = p.parse_args()

    import numpy as np
    import torch

    from hiprag import _native
    from hiprag.ivf import IvfIndex

    dev = torch.device("cuda", 0)
    N, D, B, K = args.rows, args.dim, args.batch, args.k
    st = lambda: torch.cuda.current_stream(dev).cuda_stream  # noqa: E731
    for dist in args.dist.split(","):
        if dist == "clustered":
            centers = torch.empty((args.centers, D), dtype=torch.float32, device=dev)
            _native.gen_rows_device(7, 0, args.centers, D, centers.data_ptr(), st())
            centers = torch.nn.functional.normalize(centers, dim=1)

            def rows(i0, i1):
                noise = torch.empty((i1 - i0, D), dtype=torch.float32, device=dev)
                _native.gen_rows_device(11, i0, i1 - i0, D, noise.data_ptr(), st())
                c = (torch.arange(i0, i1, device=dev, dtype=torch.int64) * 2654435761) % args.centers
                return centers[c] + args.spread * torch.nn.functional.normalize(noise, dim=1)
        else:
            def rows(i0, i1):
                x = torch.empty((i1 - i0, D), dtype=torch.float32, device=dev)
                _native.gen_rows_device(11, i0, i1 - i0, D, x.data_ptr(), st())
                return x
        t0 = time.time()
        say = lambda m: print(f"[{dist}] {m} ({time.time() - t0:.1f}s)", file=sys.stderr, flush=True)  # noqa: E731
        ivf = IvfIndex(D, args.nlist, dtype=args.dtype, metric="cosine")
        ivf.train(rows(0, min(N, args.nlist * 32)), iters=10, seed=0)
        torch.cuda.synchronize()
        say("coarse quantizer trained")
        ivf.build(N, rows)
        torch.cuda.synchronize()
        say(f"IVF lists built ({N} rows)")
        build_s = time.time() - t0
        flat = _native.NativeIndex(D, args.dtype, "cosine")
        flat.reserve(N)
        for i in range(0, N, 1 << 18):
            x = rows(i, min(N, i + (1 << 18))).contiguous()
            flat.add_device(x.data_ptr(), x.shape[0], st())
            if (i >> 18) % 64 == 63:
                say(f"exact index {i + x.shape[0]} rows")
        torch.cuda.synchronize()
        say("exact index built")
        g = torch.Generator(device=dev)
        g.manual_seed(5)
        nb = args.steps + 2
        qs = []
        for _ in range(nb):
            j = torch.randint(0, N, (B // 2,), generator=g, device=dev)
            base = torch.cat([rows(int(r), int(r) + 1) for r in j.tolist()])
            planted = base + 0.1 * torch.randn(base.shape, generator=g, device=dev)
            iso = torch.randn((B - B // 2, D), generator=g, device=dev)
            qs.append(torch.cat([planted, iso]).contiguous())
        cand = torch.empty((B, K, 2), dtype=torch.float64, device=dev)
        bound = torch.empty(B, dtype=torch.float64, device=dev)
        for i in range(2):
            ivf.search_candidates(qs[i], K, args.nprobe, cand, bound)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(2, nb):
            ivf.search_candidates(qs[i], K, args.nprobe, cand, bound)
        torch.cuda.synchronize()
        ivf_ms = (time.perf_counter() - t0) * 1e3 / args.steps
        print(f"[{dist}] IVF {ivf_ms:.3f} ms/batch", file=sys.stderr, flush=True)
        probes = torch.empty((B, args.nprobe, 2), dtype=torch.float64, device=dev)
        ivf.search_candidates(qs[2], K, args.nprobe, cand, bound, probes=probes)
        pl = probes.view(torch.int64)[..., 1]
        tiles = int((ivf.list_tiles[pl + 1] - ivf.list_tiles[pl]).sum().item())
        uniq = torch.unique(pl)
        tiles_uniq = int((ivf.list_tiles[uniq + 1] - ivf.list_tiles[uniq]).sum().item())
        esz = 4 if args.dtype == "f32" else 2
        scan_bytes, uniq_bytes = tiles * 32 * D * esz, tiles_uniq * 32 * D * esz
        ids = cand.view(torch.int64)[..., 1].cpu().numpy()
        ex_s = torch.empty((B, K), dtype=torch.float32, device=dev)
        ex_r = torch.empty((B, K), dtype=torch.int64, device=dev)
        flat.search_device(qs[2].data_ptr(), B, K, ex_s.data_ptr(), ex_r.data_ptr(), stream=st())
        torch.cuda.synchronize()
        ref = ex_r.cpu().numpy()
        t0 = time.perf_counter()
        for i in range(2, nb):
            flat.search_device(qs[i].data_ptr(), B, K, ex_s.data_ptr(), ex_r.data_ptr(), stream=st())
        torch.cuda.synchronize()
        ex_ms = (time.perf_counter() - t0) * 1e3 / args.steps

        def recall(a, b, k):
            return float(np.mean([len(set(a[i][:k]) & set(b[i][:k])) / k for i in range(len(a))]))

        h = B // 2
        print(json.dumps({
            "dist": dist, "rows": N, "dim": D, "dtype": args.dtype, "nlist": args.nlist, "nprobe": args.nprobe,
            "batch": B, "k": K, "build_s": round(build_s, 1), "ivf_ms_per_batch": round(ivf_ms, 4),
            "ivf_qps": round(B / ivf_ms * 1e3, 1), "probed_bytes_per_batch": scan_bytes,
            "distinct_probed_bytes_per_batch": uniq_bytes,
            "probed_GBps_over_batch": round(scan_bytes / (ivf_ms * 1e-3) / 1e9, 1),
            "exact_ms_per_batch": round(ex_ms, 4),
            "recall_at_100_planted": round(recall(ids[:h], ref[:h], K), 4),
            "recall_at_10_planted": round(recall(ids[:h], ref[:h], 10), 4),
            "recall_at_100_isotropic_q": round(recall(ids[h:], ref[h:], K), 4),
            "recall_at_10_isotropic_q": round(recall(ids[h:], ref[h:], 10), 4)}), flush=True)
        ivf.close()
        flat.close()
        del ivf, flat
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()

"""Shard-size sweep on one GPU: per-batch time split (scan / sample / rest) and candidates.
Usage: python tools/sweep.py [rows ...]  (dim 1024 bf16, batch 64, top-10)"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "youtu-rag_amd"), REPO]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from hiprag import _native, synth  # noqa: E402
from hiprag.dist import ShardedSearch  # noqa: E402

D, B, K = int(os.environ.get("DIM", 1024)), int(os.environ.get("BATCH", 64)), 10
sizes = [int(float(x)) for x in sys.argv[1:]] or [1_250_000, 2_500_000, 5_000_000, 10_000_000]
for n in sizes:
    idx = _native.NativeIndex(D, "bf16", "cosine")
    idx.reserve(n)
    idx.add_synthetic(0, 0, n)
    idx.set_scan_timing(1)
    qs = torch.from_numpy(np.stack([synth.planted_queries(0, n, D, B, qseed=i)[0] for i in range(13)])).cuda()
    q_ready = torch.cuda.Event()
    q_ready.record()
    ss = ShardedSearch(idx, 0, max_batch=B, overlap=os.environ.get("HIPRAG_OVERLAP", "1") != "0")
    for i in range(3):
        ss.search(qs[i], K)
    for i in range(3):  # pipelined warmup too (creates the index's pre stream outside the timed pass)
        ss.submit(qs[i], K, q_ready=q_ready)
    ss.finalize_all()
    torch.cuda.synchronize()
    idx.take_scan_times()
    cands = []
    for i in range(3, 13):  # synchronous pass: candidate counts per batch
        ss.search(qs[i], K)
        cands.append(idx.last_candidates())
    idx.take_scan_times()
    idx.set_scan_timing(8)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(3, 13):  # pipelined pass: the timed one
        ss.submit(qs[i], K, q_ready=q_ready)
    ss.finalize_all()
    torch.cuda.synchronize()
    step = (time.perf_counter() - t0) / 10 * 1e3
    samp, scan = idx.take_scan_times()
    gbs = n * D * 2 / (np.mean(scan) * 1e-3) / 1e9
    print(f"rows={n:>9} step={step:.3f}ms scan={np.mean(scan):.3f}ms ({gbs:.0f} GB/s) sample={np.mean(samp):.3f}ms "
          f"rest={step - np.mean(scan) - np.mean(samp):.3f}ms qps={B / step * 1e3:.0f} "
          f"cands/query avg={np.mean([c[0] for c in cands]) / B:.0f} max={max(c[1] for c in cands)}", flush=True)
    idx.close()
    del ss
    torch.cuda.empty_cache()

"""The query embed forward alone, for a kernel profile: bge-large shape, bf16, 64-query batches (the bench's
gpu_embed_plus_search texts), graph-replayed as the bench runs it.  Usage (GPU box):
  rocprofv3 --kernel-trace --stats -d gpurun_out/ep -- python tools/embed_prof.py [--tuned 1] [--reps 50]
Prints ms per forward (events) and the tokens per batch."""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "youtu-rag_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--tuned", type=int, default=1)
    ap.add_argument("--preset", default="bge-large")
    args = ap.parse_args()
    import torch

    from hiprag.rag.rocm_embedder import TorchRocmEmbedder

    dev = torch.device("cuda", 0)
    B = args.batch
    emb = TorchRocmEmbedder(preset=args.preset, dtype="bfloat16", batch_size=B, device=dev, seed=0,
                            tuned_gemms=bool(args.tuned))
    texts = [f"what does document {j} say about topic {j % 7} and its retrieval setup" for j in range(B)]
    for _ in range(3):
        emb.embed_queries_device(texts)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    t0 = time.perf_counter()
    for _ in range(args.reps):
        emb.embed_queries_device(texts)
    e1.record()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    toks = emb.tokenizer(texts, padding=True, truncation=True, return_tensors="pt", max_length=emb.max_length)
    print(json.dumps({"ms_per_forward_events": round(e0.elapsed_time(e1) / args.reps, 4),
                      "ms_per_forward_wall": round(1000 * dt / args.reps, 4), "tuned": emb.tuned_gemms,
                      "graphs": len(emb.graphed.graphs) if emb.graphed else 0,
                      "tokens_per_batch": int(toks["attention_mask"].sum())}))


if __name__ == "__main__":
    main()

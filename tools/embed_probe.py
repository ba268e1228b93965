"""Where the query embed's time goes (bench.py gpu_embed_plus_search): host tokenisation, host dispatch of the
unpadded forward, and the forward's GPU time; then the same forward captured once in a HIP graph and replayed.
Usage (GPU box): python tools/embed_probe.py [--batches 16]"""
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
    ap.add_argument("--batches", type=int, default=16)
    ap.add_argument("--batch", type=int, default=64)
    args = ap.parse_args()
    import torch

    from hiprag.rag.rocm_embedder import TorchRocmEmbedder

    dev = torch.device("cuda", 0)
    B = args.batch
    emb = TorchRocmEmbedder(preset="bge-large", dtype="bfloat16", batch_size=B, device=dev, seed=0)
    texts = [[f"what does document {i * B + j} say about topic {(i * B + j) % 7} and its retrieval setup"
              for j in range(B)] for i in range(args.batches + 2)]
    out = {}
    for t in texts[:2]:
        emb.embed_queries_device(t)
    torch.cuda.synchronize()
    # 1. host tokenisation alone
    t0 = time.perf_counter()
    toks = [emb.tokenizer(t, padding=True, truncation=True, return_tensors="pt", max_length=emb.max_length,
                          add_special_tokens=True) for t in texts[2:]]
    out["tokenize_ms"] = round(1000 * (time.perf_counter() - t0) / args.batches, 3)
    # 2. pack + forward: host time to enqueue, GPU time by events
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    host, gpu = [], []
    with torch.inference_mode():
        for b in toks:
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            pk = emb.unpadded.pack([b["input_ids"]], [b["attention_mask"]], [b.get("token_type_ids")])
            e0.record()
            h = emb.unpadded.forward_packed(pk)
            e1.record()
            host.append(time.perf_counter() - t0)
            torch.cuda.synchronize()
            gpu.append(e0.elapsed_time(e1))
    out["pack_plus_dispatch_host_ms"] = round(1000 * sum(host) / len(host), 3)
    out["forward_gpu_ms_events"] = round(sum(gpu) / len(gpu), 3)
    out["tokens_per_batch"] = int(toks[0]["attention_mask"].sum())
    # 3. the same forward captured in a graph (fixed packed shape), replayed
    try:
        with torch.inference_mode():
            b = toks[0]
            pk = emb.unpadded.pack([b["input_ids"]], [b["attention_mask"]], [b.get("token_type_ids")])
            s = torch.cuda.Stream(dev)
            s.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(s):
                for _ in range(2):
                    emb.unpadded.forward_packed(pk)
            torch.cuda.current_stream(dev).wait_stream(s)
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                hg = emb.unpadded.forward_packed(pk)
            torch.cuda.synchronize()
            ref = emb.unpadded.forward_packed(pk)
            g.replay()
            torch.cuda.synchronize()
            out["graph_max_abs_diff"] = float((hg.float() - ref.float()).abs().max())
            t0 = time.perf_counter()
            for _ in range(args.batches):
                g.replay()
            torch.cuda.synchronize()
            out["graph_replay_ms"] = round(1000 * (time.perf_counter() - t0) / args.batches, 3)
    except Exception as e:  # noqa: BLE001 -- a probe: report what failed
        out["graph_error"] = f"{type(e).__name__}: {e}"[:300]
    print(json.dumps(out))


if __name__ == "__main__":
    main()

"""Tune the encoder GEMMs with torch TunableOp (every hipBLASLt / rocBLAS solution of a shape benchmarked, the
fastest kept) for the token counts the graph-replayed forward runs at (multiples of 64, GraphedForward's granule),
and write the results file the embedder loads read-only (hiprag/rag/tunableop_gfx950.csv).  Then time the query
embed (bge-large shape, bf16, B = 64) with the heuristic choice and with the tuned one.
Usage (GPU box): python tools/embed_tune.py --out F [--max-tokens 8192] [--presets bge-large,bge-base]"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "youtu-rag_amd"))


def timed(emb, texts, torch):
    for t in texts[:2]:
        emb.embed_queries_device(t)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    outs = [emb.embed_queries_device(t) for t in texts]
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / len(texts), outs


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", required=True)
    ap.add_argument("--max-tokens", type=int, default=8192)
    ap.add_argument("--presets", default="bge-large,bge-base")
    ap.add_argument("--batches", type=int, default=16)
    args = ap.parse_args()
    import torch
    import torch.cuda.tunable as tun

    from hiprag.rag.rocm_embedder import PRESETS, TorchRocmEmbedder

    dev = torch.device("cuda", 0)
    B = 64
    texts = [[f"what does document {i * B + j} say about topic {(i * B + j) % 7} and its retrieval setup"
              for j in range(B)] for i in range(args.batches)]
    res = {}
    emb = TorchRocmEmbedder(preset="bge-large", dtype="bfloat16", batch_size=B, device=dev, seed=0, tuned_gemms=False)
    res["default_ms"], ref = timed(emb, texts, torch)
    del emb
    torch.cuda.synchronize()
    # tune: the four GEMMs of an encoder layer (QKV, attention output, intermediate, output) with bias, bf16, at
    # every token count that is a multiple of 64
    tun.set_filename(args.out)
    tun.enable(True)
    tun.tuning_enable(True)
    t0 = time.perf_counter()
    for name in args.presets.split(","):
        H, inter = PRESETS[name]["hidden_size"], PRESETS[name]["intermediate_size"]
        for n_out, k_in in ((3 * H, H), (H, H), (inter, H), (H, inter)):
            w = torch.randn(n_out, k_in, device=dev, dtype=torch.bfloat16)
            b = torch.randn(n_out, device=dev, dtype=torch.bfloat16)
            for m in range(64, args.max_tokens + 1, 64):
                x = torch.randn(m, k_in, device=dev, dtype=torch.bfloat16)
                torch.nn.functional.linear(x, w, b)
        torch.cuda.synchronize()
    res["tuning_s"] = round(time.perf_counter() - t0, 1)
    tun.tuning_enable(False)
    res["results"] = len(tun.get_results())
    tun.enable(False)
    emb = TorchRocmEmbedder(preset="bge-large", dtype="bfloat16", batch_size=B, device=dev, seed=0, tuned_gemms=True)
    res["tuned_ms"], got = timed(emb, texts, torch)
    res["max_abs_diff_vs_default"] = max(float((a.float() - b.float()).abs().max()) for a, b in zip(got, ref))
    res = {k: (round(v * 1000, 3) if k.endswith("_ms") else v) for k, v in res.items()}
    print(json.dumps(res))


if __name__ == "__main__":
    main()

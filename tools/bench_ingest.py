"""Config 4 (BASELINE.json configs[3]): end-to-end KB ingest on one MI355X.

synthetic documents -> RecursiveTextSplitter (chunk 500 / overlap 50, agent.py:172-173)
-> TorchRocmEmbedder (random-init BERT of the named preset; PyTorch-ROCm forward + K7)
-> hr_index_add_device -> batched query (embed + search).  Prints one JSON line:
chunks/s for the whole ingest, the per-stage split, query latency, and a CPU leg
(the same embedder forward on the host cores for a bounded sample -- the reference's
server on a CPU box; `cores` = torch threads).  Data: synthetic text (no corpus offline),
random-init weights (no checkpoints offline).

    python tools/bench_ingest.py --chunks 100000 --preset bge-large --dtype bfloat16
"""
from __future__ import annotations

import argparse
import asyncio
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "youtu-rag_amd")]


def make_docs(n_chunks: int, seed: int = 0):
    import numpy as np

    from hiprag.rag import Document

    rng = np.random.default_rng(seed)
    vocab = [f"w{i}" for i in range(20000)]
    p = 1.0 / np.arange(1, len(vocab) + 1)
    p /= p.sum()
    # ~10 chunks of 500 characters per document
    docs, per_doc = [], 4500
    n_docs = max(1, n_chunks // 10)
    for d in range(n_docs):
        words = rng.choice(len(vocab), size=per_doc // 5, p=p)
        sents = [" ".join(vocab[w] for w in words[i:i + 14]) for i in range(0, len(words), 14)]
        docs.append(Document(id=f"doc{d}.pdf", content=". ".join(sents), metadata={"source": f"kb/doc{d}.pdf"}))
    return docs


def cpu_embed_rate(preset: str, texts: list[str], max_length: int, batch: int = 16) -> float:
    """The reference server's encode (mdx:81-116) on the host cores: fp32 forward, torch pooling."""
    import torch

    from hiprag.rag.rocm_embedder import HashWordTokenizer, build_random_bert

    model = build_random_bert(preset, 0).eval()
    tok = HashWordTokenizer()
    t = time.perf_counter()
    with torch.inference_mode():
        for i in range(0, len(texts), batch):
            inp = tok(texts[i:i + batch], padding=True, truncation=True, max_length=max_length, return_tensors="pt")
            h = model(**inp)[0]
            m = inp["attention_mask"].clone()
            m[:, :2] = 0
            e = (h * m.unsqueeze(-1).float()).sum(1) / m.sum(1, keepdim=True).float()
            torch.nn.functional.normalize(e, dim=-1)
    return len(texts) / (time.perf_counter() - t)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--chunks", type=int, default=100_000)
    ap.add_argument("--preset", default="bge-base", help="bge-base (SURVEY §8(d) C4: 12 layers, H = 768) or bge-large")
    ap.add_argument("--dtype", default="bfloat16")
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--max-length", type=int, default=512)
    ap.add_argument("--queries", type=int, default=64)
    ap.add_argument("--cpu-sample", type=int, default=64)
    ap.add_argument("--stages", action="store_true",
                    help="time split / embed / add separately (synchronises around each stage: no overlap)")
    args = ap.parse_args()

    import torch

    from hiprag.rag import BatchedVectorRetriever, ChunkingConfig, HipVectorStore, RetrieverConfig, VectorStoreConfig
    from hiprag.rag.ingest import GpuIngestor
    from hiprag.rag.rocm_embedder import TorchRocmEmbedder

    t0 = time.perf_counter()
    docs = make_docs(args.chunks)
    splitter_cfg = ChunkingConfig(chunk_size=500, chunk_overlap=50)
    t_gen = time.perf_counter() - t0
    emb = TorchRocmEmbedder(preset=args.preset, dtype=args.dtype, batch_size=args.batch, max_length=args.max_length)
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from flops import EncoderFlops, mfma_block

    counter = EncoderFlops(emb.model, getattr(emb, "unpadded", None))
    store = HipVectorStore(VectorStoreConfig(backend="hip", collection_name="bench", persist_directory="/tmp/unused",
                                             index_params={"dtype": "bf16", "persist": False,
                                                           "capacity": int(args.chunks * 1.2)}))
    ing = GpuIngestor(store, emb, chunking=splitter_cfg)

    stage = {"split_s": 0.0, "embed_s": 0.0, "tokenize_s": 0.0, "add_s": 0.0}  # tokenize_s is inside embed_s
    tok_inner = emb.tokenizer

    def timed_tok(*a, **k):
        t = time.perf_counter()
        r = tok_inner(*a, **k)
        stage["tokenize_s"] += time.perf_counter() - t
        return r

    emb.tokenizer = timed_tok
    inner_embed, inner_add, inner_split = emb.embed_texts_device, store.add_chunks_device, ing.split

    def embed(texts):
        torch.cuda.synchronize()
        t = time.perf_counter()
        out = inner_embed(texts)
        torch.cuda.synchronize()
        stage["embed_s"] += time.perf_counter() - t
        return out

    def add(chunks, e):
        t = time.perf_counter()
        r = inner_add(chunks, e)
        stage["add_s"] += time.perf_counter() - t
        return r

    def split(d, m=None):
        t = time.perf_counter()
        r = inner_split(d, m)
        stage["split_s"] += time.perf_counter() - t
        return r

    if args.stages:
        emb.embed_texts_device, store.add_chunks_device, ing.split = embed, add, split
    # warm-up (kernel selection, allocator) on a few documents, then a clean store
    asyncio.run(ing.ingest(docs[:3]))
    asyncio.run(store.clear())
    for k in stage:
        stage[k] = 0.0
    counter.reset()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    last = t0
    n_chunks = 0
    step = max(1, len(docs) // 20)
    for i in range(0, len(docs), step):
        n_chunks += asyncio.run(ing.ingest(docs[i:i + step]))
        if time.perf_counter() - last > 30:
            last = time.perf_counter()
            print(f"[ingest] {n_chunks} chunks, {last - t0:.1f}s", file=sys.stderr, flush=True)
    torch.cuda.synchronize()
    t_ing = time.perf_counter() - t0
    flops = counter.totals()
    # queries: embed + one batched search
    ret = BatchedVectorRetriever(store, emb, RetrieverConfig(top_k=10, similarity_threshold=0.0))
    qs = [" ".join(d.content.split()[5:15]) for d in docs[:args.queries]]
    asyncio.run(ret.batch_retrieve(qs, top_k=10))
    torch.cuda.synchronize()
    t = time.perf_counter()
    res = asyncio.run(ret.batch_retrieve(qs, top_k=10))
    torch.cuda.synchronize()
    t_q = time.perf_counter() - t
    hit = sum(1 for r in res if r)
    # CPU leg: the same forward on the host cores for a bounded sample
    threads = int(os.environ.get("OMP_NUM_THREADS", "16"))
    torch.set_num_threads(threads)
    texts = [c.content for c in inner_split(docs[0])] * (1 + args.cpu_sample // 8)
    texts = texts[:args.cpu_sample]
    cpu_rate = cpu_embed_rate(args.preset, texts, args.max_length)
    print(json.dumps({
        "metric": "KB ingest chunks/s (split -> embed -> index), 1 MI355X", "value": round(n_chunks / t_ing, 1),
        "unit": "chunks/s", "chunks": n_chunks, "ingest_s": round(t_ing, 2), "stages": {k: round(v, 2) for k, v in stage.items()},
        "query_batch": args.queries, "query_batch_ms": round(t_q * 1e3, 2), "queries_answered": hit,
        "dtype": args.dtype, "data": "synthetic text, random-init weights",
        "config": {"workload": "C4 ingest", "preset": args.preset, "batch": args.batch, "max_length": args.max_length,
                   "chunk_size": 500, "chunk_overlap": 50, "docgen_s": round(t_gen, 2)},
        # the embedder against the MFMA roof: encoder FLOPs over the whole ingest's wall time (split, tokenise,
        # forward, pool, add pipelined); with --stages over the embed stage's own time
        "mfma": mfma_block(flops, stage["embed_s"] if args.stages else t_ing,
                           what="embedder forward FLOPs (tools/flops.py) per second of "
                                + ("the embed stage" if args.stages else "the whole ingest")),
        "cpu_baseline": {"value": round(cpu_rate, 2), "unit": "chunks/s (embed only)", "cores": threads,
                         "kind": "port", "sample": f"{len(texts)} chunks, same model fp32 on host torch"},
    }), flush=True)


if __name__ == "__main__":
    main()

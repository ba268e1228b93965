#!/usr/bin/env python3
"""Headline benchmark: brute-force exact top-k retrieval QPS over a row-sharded corpus.

BASELINE.json metric: "retrieval QPS + recall@10 vs CPU ref, 10M×1024 corpus, 1/2/4/8 MI355X".
Workload (configs[2], which fits one MI355X: 20.5 GB of bf16): 10M × 1024 bf16 chunk
vectors, cosine, top-10, batches of 64 queries, corpus row-sharded over the ranks
(strong scaling: the corpus is fixed, each of G ranks holds N/G rows).  A "step" is
one batch of 64 queries through the whole distributed path: per-shard MFMA scan +
exact rescoring, RCCL all-gather of candidates, exact merge, guard/fallback.

Launch: python bench.py [--gpus N --steps K --warmup W]; for N > 1 under
torch.distributed.run (one rank per GPU, RCCL).  Rank 0 prints ONE JSON line.

Inputs are resident in HBM before the timed region: every rank generates its shard
on its GPU with the counter-based generator (hiprag.synth) and all query batches
are uploaded up front.  ``cpu_baseline`` (rank 0, N=1 only) times the reference's CPU
search path (FAISS IndexFlatIP semantics = BLAS sgemm + top-k over the fp32 store, its
per-query loop and the CPU query embedding) on a bounded row sample and scales it to the
full corpus; ``cpu_oracle`` times the exact fp64 checker (oracle/, test infrastructure);
``recall_at_10`` compares the GPU's first batch with the oracle's exact answer over the
FULL corpus for a few queries.  ``--single-process`` runs one process with one index handle
striped over the GPUs instead (hr_index_create with n_dev > 1).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "youtu-rag_amd"))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402

METRIC = "retrieval QPS + recall@10 vs CPU ref, 10M×1024 corpus, 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec (6.29 TB/s measured float4 copy)
# the practical read ceiling: a read-only kernel with the scan's access shape and launch (n_cu - 32 CUs,
# 8 waves/CU, non-temporal 16 B lane loads) over 20.48 GB, tools/stream_ceiling.hip ->
# profiles/r02_stream_ceiling.jsonl ("nt, n_cu-32 CUs, 8 waves/CU (the scan's launch)")
HBM_READ_CEILING_GBS = 7076.6
MFMA_PEAK_TFLOPS = 2500.0  # dense bf16 (no sparsity), MI355X_MICROARCH.md


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=200)
    p.add_argument("--warmup", type=int, default=10)
    p.add_argument("--rows", type=int, default=10_000_000)
    p.add_argument("--dim", type=int, default=1024)
    p.add_argument("--batch", type=int, default=64)
    p.add_argument("--k", type=int, default=10)
    p.add_argument("--dtype", default="bf16")
    p.add_argument("--seed", type=int, default=0)
    p.add_argument("--cpu-sample-rows", type=int, default=2_000_000)
    p.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU search time the cpu_baseline accumulates")
    p.add_argument("--cpu-ref-rows", type=int, default=1_000_000, help="row sample of the reference-path CPU baseline")
    p.add_argument("--cpu-embed-preset", default="bge-large")
    p.add_argument("--recall-queries", type=int, default=64, help="planted and isotropic queries of the recall checks")
    p.add_argument("--no-cpu", action="store_true", help="skip cpu_baseline, recall and the GPU embed leg (quick runs)")
    p.add_argument("--no-embed", action="store_true", help="skip the GPU embed+search leg")
    # (off by default: with the CUs split 48/64/96/128 : rest the pipeline measured 5.4k / 6.6k / 7.0k / 7.0k QPS
    # against 9.1k sharing every CU and 9.8k sequential -- profiles/r05_embed_cu_split.json)
    p.add_argument("--embed-cus", default="",
                   help="CU shares of the query embedder in the embed+search leg's CU-split runs, e.g. 64,96 ('' = none)")
    p.add_argument("--launch-probe", action="store_true", help=argparse.SUPPRESS)  # tests: launcher only
    p.add_argument("--collective", action="store_true",
                   help="run the exchange through an RCCL process group even at --gpus 1 (world size 1): the timed "
                        "loop then includes the all-gather an 8-GPU node runs")
    p.add_argument("--persist", type=int, default=1, choices=(0, 1, 2),
                   help="persistent FILTER for the pipelined shard batches: 0 off (one FILTER launch per batch), "
                        "1 shards of 4.2M-5.1M rows (default: where it measured faster), 2 every shard size")
    p.add_argument("--q256", type=int, default=1, choices=(0, 1),
                   help="129-256-query batches: the 256-query FILTER (1, default) or two 128-query FILTER launches (0)")
    p.add_argument("--depth", type=int, default=2,
                   help="batches in flight per rank (ShardedSearch depth): the host waits for batch i's guard flags "
                        "when it submits batch i + depth")
    p.add_argument("--single-process", action="store_true",
                   help="one process, one index handle striped over --gpus devices (instead of one rank per GPU)")
    return p.parse_args()


def log(*a):
    print(*a, file=sys.stderr, flush=True)


TIME_EVERY = 8


def summary_order(path: str):
    """Sort key of a committed profile summary, oldest first: round number, then the tag's trailing sequence number
    (r04final3 after r04final), then the summary's own creation stamp (tools/summarize_profile.py, round 5 on).
    Lexical order put r04final3_... BEFORE r04final_... ('3' < '_'), so the bench cited a stale summary (VERDICT
    r04 weak #6)."""
    import re

    name = os.path.basename(path)
    m = re.match(r"r(\d+)([A-Za-z]*)(\d*)_", name)
    rnd, seq = (int(m.group(1)), int(m.group(3) or 0)) if m else (-1, 0)
    created = ""
    try:
        with open(path) as f:
            created = str(json.load(f).get("created_utc", ""))
    except (OSError, ValueError):
        pass
    return rnd, seq, created, name


def cpu_reference_baseline(args, qbatches, N, D, K, B):
    """The reference's CPU search path timed on the host cores, on a bounded row sample.

    (b) ``value``: FAISSVectorStore.search over its fp32 store (faiss_store.py:98, :148-154:
        normalize_L2(query) + IndexFlatIP.search = one sgemm of the query batch against the rows +
        a top-k selection), restated with numpy's BLAS sgemm + argpartition over 128k-row blocks,
        a whole 64-query batch per call -- the CPU's best case;
    (a) ``per_query_loop``: VectorRetriever.batch_retrieve's sequential loop (base_retriever.py:
        96-98): one sgemv + selection per query, as the reference issues them;
    ``embed``: the embedding server's encode (deploying-locally.mdx:81-116: tokenise, transformer
        forward, instruction-masked mean-pool, L2 normalise) of one query per call on the same
        cores, for the north_star's "CPU embed+search" figure (random-init bge-large, no weights
        offline).
    Rows: the synthetic corpus (the same generator), normalised, bf16-quantised like the GPU store,
    held as fp32 as the reference store holds them.  Scaled by N / sample rows."""
    import oracle
    from oracle import ref_numpy as R

    threads = oracle.default_threads()
    try:
        from threadpoolctl import threadpool_info

        blas = [{"api": p.get("internal_api"), "threads": p.get("num_threads")} for p in threadpool_info()
                if p.get("user_api") == "blas"]
    except Exception:  # noqa: BLE001
        blas = []
    S = min(args.cpu_ref_rows, N)
    x = R.dequantize(oracle.c_build_synthetic(args.seed, 0, S, D, args.dtype, "cosine", threads), args.dtype)
    blk = 1 << 17

    def search(qn, k):
        best_s = np.full((len(qn), k), -np.inf, np.float32)
        best_r = np.full((len(qn), k), -1, np.int64)
        for r0 in range(0, S, blk):
            sc = qn @ x[r0:r0 + blk].T                                   # IndexFlatIP: sgemm / sgemv
            kk = min(k, sc.shape[1])
            idx = np.argpartition(-sc, kk - 1, axis=1)[:, :kk]
            all_s = np.concatenate([best_s, np.take_along_axis(sc, idx, 1)], 1)
            all_r = np.concatenate([best_r, idx + r0], 1)
            o = np.argsort(-all_s, axis=1, kind="stable")[:, :k]
            best_s, best_r = np.take_along_axis(all_s, o, 1), np.take_along_axis(all_r, o, 1)
        return best_s, best_r

    def normalize(q):  # faiss.normalize_L2
        q = np.asarray(q, np.float32)
        return q / np.linalg.norm(q, axis=1, keepdims=True)

    search(normalize(qbatches[0][:2]), K)  # warm the BLAS threads
    dt, nb = 0.0, 0
    while nb < len(qbatches) and (dt < args.cpu_seconds or nb == 0):
        t1 = time.perf_counter()
        search(normalize(qbatches[nb]), K)
        dt += time.perf_counter() - t1
        nb += 1
    qps_b = nb * B / (dt * (N / S))
    # (a) one query per call
    nq, ta = 0, 0.0
    flat = np.concatenate(qbatches[:2])
    while nq < len(flat) and (ta < args.cpu_seconds / 3 or nq == 0):
        t1 = time.perf_counter()
        search(normalize(flat[nq:nq + 1]), K)
        ta += time.perf_counter() - t1
        nq += 1
    qps_a = nq / (ta * (N / S))
    out = {"value": round(qps_b, 3), "unit": "queries/s", "cores": threads, "kind": "port",
           "path": "FAISSVectorStore.search semantics (faiss_store.py:148-154: normalize_L2 + IndexFlatIP = sgemm + "
                   "top-k) over the fp32 store, numpy BLAS",
           "sample": f"{nb} batches x {B} queries over {S} of the {N} rows ({dt:.2f}s), scaled by {N / S:.1f}x",
           "blas": blas,
           "per_query_loop": {"value": round(qps_a, 3), "unit": "queries/s",
                              "path": "VectorRetriever.batch_retrieve's per-query loop (base_retriever.py:96-98): "
                                      "one sgemv + top-k per query",
                              "sample": f"{nq} queries over {S} rows ({ta:.2f}s), scaled by {N / S:.1f}x"}}
    del x
    # CPU query embedding (the server's encode on the host cores, one query per call)
    try:
        import torch

        from hiprag.rag.rocm_embedder import DEFAULT_QUERY_INSTRUCTION, HashWordTokenizer, build_random_bert

        torch.set_num_threads(threads)
        model = build_random_bert(args.cpu_embed_preset, seed=0).eval()
        tok = HashWordTokenizer()
        instr = f"Instruction: {DEFAULT_QUERY_INSTRUCTION} \nQuery:"
        n_instr = len(tok(instr, add_special_tokens=True)["input_ids"])
        queries = [f"what does document {i} say about topic {i % 7} and its retrieval setup" for i in range(6)]

        def encode(q):
            inp = tok([instr + q], padding=True, truncation=True, max_length=512, return_tensors="pt")
            with torch.inference_mode():
                h = model(**inp)[0]
                m = inp["attention_mask"].clone()
                m[:, :n_instr] = 0
                v = (h * m[..., None]).sum(1) / m.sum(1, keepdim=True)
                return torch.nn.functional.normalize(v, dim=-1)

        encode(queries[0])
        te, ne = 0.0, 0
        for q in queries[1:]:
            t1 = time.perf_counter()
            encode(q)
            te += time.perf_counter() - t1
            ne += 1
        ms = 1000.0 * te / ne
        out["embed"] = {"ms_per_query": round(ms, 2), "model": f"{args.cpu_embed_preset} (random init), fp32",
                        "queries": ne}
        out["embed_plus_search_per_query_qps"] = round(1.0 / (ms / 1000.0 + 1.0 / qps_a), 4)
        out["embed_plus_search_batched_qps"] = round(1.0 / (ms / 1000.0 + 1.0 / qps_b), 4)
    except Exception as e:  # noqa: BLE001
        out["embed"] = {"error": repr(e)}
    return out


def gpu_embed_plus_search(args, searcher, dev, D, K, B, n_batches: int = 16) -> dict:
    """The reference's query path on the GPU, beside cpu_baseline's CPU embed+search: ``embed_query`` then
    ``search`` (base_retriever.py:57-62; the embedding server's encode, deploying-locally.mdx:81-116) -- B query
    strings -> TorchRocmEmbedder (the same bge-large shape as the CPU leg, bf16, unpadded packed forward replayed
    from HIP graphs + K7 pooling) -> the exact scan over the resident corpus (this bench's searcher), timed end to
    end:
    * ``sequential``: one batch at a time, embed -> search -> synchronise (a lone caller's latency);
    * ``pipelined``: the embedder on a stream of its own, each batch's search submitted behind its queries' event,
      two batches in flight (the throughput a serving process gets);
    plus the embed alone and its MFMA rate (executed FLOPs of the forwards ÷ time, against the 2.5 PF bf16 peak).
    Random-init weights (no checkpoint offline), so the vectors are not semantically meaningful: the figure is
    the work's cost, not retrieval quality."""
    import torch

    from hiprag.rag.rocm_embedder import TorchRocmEmbedder

    sys.path.insert(0, os.path.join(REPO, "tools"))
    from flops import EncoderFlops

    emb = TorchRocmEmbedder(preset=args.cpu_embed_preset, dtype="bfloat16", batch_size=B, device=dev, seed=0,
                            tuned_gemms=True)  # (the shipped gfx950 GEMM results: an application opt-in)
    if emb.dim != D:
        return {"skipped": f"embedder dim {emb.dim} != corpus dim {D}"}
    fl = EncoderFlops(emb.model, emb.unpadded)
    texts = [[f"what does document {i * B + j} say about topic {(i * B + j) % 7} and its retrieval setup"
              for j in range(B)] for i in range(n_batches + 2)]
    # warm: kernels, allocator, tokenizer caches and the embed's HIP graphs -- one per packed shape (a serving
    # process's steady state: query batches fall into a few shapes, each captured once; encoder.GraphedForward)
    for t in texts:
        searcher.search(emb.embed_queries_device(t), K)
    torch.cuda.synchronize()
    fl.reset()
    t0 = time.perf_counter()
    for t in texts[2:]:
        emb.embed_queries_device(t)
    torch.cuda.synchronize()
    t_embed = (time.perf_counter() - t0) / n_batches
    flops = fl.totals()
    t0 = time.perf_counter()
    for t in texts[2:]:
        searcher.search(emb.embed_queries_device(t), K)
        torch.cuda.synchronize()
    t_seq = (time.perf_counter() - t0) / n_batches
    es = torch.cuda.Stream(dev)
    s_out = torch.empty((n_batches, B, K), dtype=torch.float32, device=dev)
    r_out = torch.empty((n_batches, B, K), dtype=torch.int64, device=dev)
    keep = []
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i, t in enumerate(texts[2:]):
        with torch.cuda.stream(es):
            q = emb.embed_queries_device(t)
            ev = torch.cuda.Event()
            ev.record(es)
        keep.append((q, ev))
        torch.cuda.current_stream(dev).wait_event(ev)  # (the scan stream's own order: prep runs behind the queries)
        searcher.submit(q, K, s_out=s_out[i], r_out=r_out[i], q_ready=ev)
    searcher.finalize_all()
    torch.cuda.synchronize()
    t_pipe = (time.perf_counter() - t0) / n_batches
    tflops = flops["executed"] / n_batches / t_embed / 1e12
    # the same pipeline with the GPU split by CU (VERDICT r04 missing #4): the compute-bound forward on its own CUs
    # (a CU-masked stream), the HBM-bound scan -- prep, SAMPLE, FILTER, select, rescore, merge -- on the others
    # (hr_index_set_cu_mask for the index's streams, masked scan / tail streams for ShardedSearch), so the two
    # overlap instead of contending for every CU
    split = {}
    q_last = keep[-1][0].float().cpu().numpy()  # the last batch's embedded queries (shared-CU run)
    if args.embed_cus:
        split = embed_search_cu_split(args, searcher, emb, texts[2:], dev, K, B, s_out, r_out)
    best = min([(t_pipe, None)] + [(v["ms_per_batch"] / 1e3, n) for n, v in split.items()])
    # the embedded queries' answers against the oracle over all rows (the last batch, as the pipelined runs left it)
    import oracle
    from oracle import ref_numpy as R

    s_ref, r_ref = oracle.c_search_synthetic(args.seed, 0, args.rows, D, args.dtype, "cosine",
                                             R.process_queries(q_last, "cosine"), K)
    oracle_ok = bool(np.array_equal(r_out[-1].cpu().numpy(), r_ref)
                     and np.array_equal(s_out[-1].cpu().numpy(), s_ref.astype(np.float32)))
    return {"model": f"{args.cpu_embed_preset} shape (random init), bf16, unpadded forward + K7", "batch": B,
            "batches": n_batches, "tokens_per_batch": round(flops["tokens_real"] / n_batches, 1),
            "embed_ms_per_batch": round(1000 * t_embed, 3), "embed_tflops": round(tflops, 1),
            "embed_graphs": len(emb.graphed.graphs) if emb.graphed is not None else 0,
            "embed_frac_of_bf16_peak": round(tflops / MFMA_PEAK_TFLOPS, 4),
            "sequential": {"ms_per_batch": round(1000 * t_seq, 3), "qps": round(B / t_seq, 1)},
            "pipelined": {"ms_per_batch": round(1000 * best[0], 3), "qps": round(B / best[0], 1),
                          "embed_cus": best[1], "shared_cus_ms_per_batch": round(1000 * t_pipe, 3)},
            "pipelined_cu_split": split,
            "last_batch_ids_identical_to_oracle": oracle_ok,
            "path": "embed_query -> search (base_retriever.py:57-62), embedding + exact scan on the GPU"}


def embed_search_cu_split(args, searcher, emb, texts, dev, K, B, s_out, r_out) -> dict:
    """gpu_embed_plus_search's pipelined leg with the CUs partitioned: for each embed share n in --embed-cus, the
    embedder runs on a stream masked to n CUs spread evenly over the chip (CU i with i * n // n_cu stepping), and the
    index's internal streams plus ShardedSearch's scan and tail streams on the rest.  Every batch's answers are
    checked against the shared-CU run's (same embeddings, so identical ids and scores).  Returns
    {n: {ms_per_batch, qps}}."""
    import torch

    from hiprag import _native

    n_cu = torch.cuda.get_device_properties(dev).multi_processor_count
    ref_s, ref_r = s_out.clone(), r_out.clone()
    out = {}
    for n in (int(x) for x in args.embed_cus.split(",")):
        if not 16 <= n <= n_cu - 48:
            continue
        e_cus = sorted({(i * n_cu) // n for i in range(n)})
        s_cus = [c for c in range(n_cu) if c not in set(e_cus)]
        raw = [_native.create_cu_stream(dev.index or 0, e_cus), _native.create_cu_stream(dev.index or 0, s_cus),
               _native.create_cu_stream(dev.index or 0, s_cus)]
        es, scan, tail = (torch.cuda.ExternalStream(r, device=dev) for r in raw)
        tail0 = searcher.tail
        try:
            searcher.index.set_cu_mask(s_cus)
            searcher.tail = tail
            keep = []
            for rep in range(2):  # (the first pass warms the masked streams)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for i, t in enumerate(texts):
                    with torch.cuda.stream(es):
                        q = emb.embed_queries_device(t)
                        ev = torch.cuda.Event()
                        ev.record(es)
                    keep.append((q, ev))
                    scan.wait_event(ev)
                    with torch.cuda.stream(scan):
                        searcher.submit(q, K, s_out=s_out[i], r_out=r_out[i], q_ready=ev)
                searcher.finalize_all()
                torch.cuda.synchronize()
                dt = (time.perf_counter() - t0) / len(texts)
            ok = bool(torch.equal(s_out, ref_s) and torch.equal(r_out, ref_r))
            out[str(n)] = {"ms_per_batch": round(1000 * dt, 3), "qps": round(B / dt, 1), "search_cus": len(s_cus),
                           "results_identical_to_shared": ok}
        finally:
            searcher.finalize_all()
            torch.cuda.synchronize()
            searcher.tail = tail0
            searcher.index.set_cu_mask(None)
            for r in raw:  # (nothing of torch's remembers them: the search copies its flags through the library)
                _native.destroy_stream(r)
    return out


def isotropic_queries(B: int, D: int, seed: int = 7) -> np.ndarray:
    """B isotropic Gaussian queries: no planted neighbour, so every top-k score sits in the dense upper
    tail of the corpus' score distribution -- the smallest gaps between ranks, the hardest case for a
    quantised store's ranking."""
    return np.random.default_rng(seed).standard_normal((B, D)).astype(np.float32)


def recall_checks(args, N, D, K, q_pl, got_pl, s_pl, q_iso, got_iso, s_iso) -> dict:
    """The GPU's top-k against the CPU oracle over ALL N rows, for planted and isotropic queries:
    (i) ``ids_identical`` / ``recall_at_10`` / ``max_score_err`` -- against the exact answer over the rows
    as the GPU stores them (args.dtype): the parity claim (bit-exact ids, scores within 0);
    (ii) ``recall_at_10_vs_fp32`` -- against the exact answer over the UNQUANTISED fp32 rows, which is
    what the reference's store holds (faiss_store.py:98, normalize_L2 + IndexFlatIP over float32): how far
    a bf16 store's ranking departs from the reference's answers."""
    import oracle
    from oracle import ref_numpy as R

    out = {}
    t1 = time.time()
    qn = R.process_queries(np.concatenate([q_pl, q_iso]), "cosine")
    got = np.concatenate([got_pl, got_iso])
    s_gpu = np.concatenate([s_pl, s_iso])
    n_pl = len(q_pl)

    def rec(a, b):
        return float(np.mean([len(set(a[i]) & set(b[i])) / K for i in range(len(a))]))

    s_ref, r_ref = oracle.c_search_synthetic(args.seed, 0, N, D, args.dtype, "cosine", qn, K)
    out["recall_at_10"] = rec(got[:n_pl], r_ref[:n_pl])
    out["ids_identical"] = bool(np.array_equal(got, r_ref))
    out["max_score_err"] = float(np.max(np.abs(s_gpu - s_ref.astype(np.float32))))
    out["recall_check"] = (f"{n_pl} planted + {len(q_iso)} isotropic queries (first timed batch / one extra batch) "
                           f"vs the CPU oracle over all {N} rows as stored ({args.dtype})")
    if args.dtype != "f32":
        _, r32 = oracle.c_search_synthetic(args.seed, 0, N, D, "f32", "cosine", qn, K)
        out["recall_at_10_vs_fp32"] = {
            "planted": rec(got[:n_pl], r32[:n_pl]), "isotropic": rec(got[n_pl:], r32[n_pl:]),
            "top1_agree": float(np.mean(got[:, 0] == r32[:, 0])),
            "reference": f"exact top-{K} over the unquantised fp32 rows (the reference store's dtype), "
                         f"{n_pl} planted + {len(q_iso)} isotropic queries"}
    log(f"recall checks {time.time() - t1:.1f}s")
    return out


def main_single_process(args):
    """--single-process: ONE process, ONE index handle over --gpus devices (hr_index_create with
    n_dev > 1: rows striped over the GPUs by tile, per-shard scans on every device at once, the
    candidates peer-copied to device 0 and merged there) -- the reference's deployment shape (one
    FastAPI process, one store per collection).  Batches are pipelined through hr_index_search_submit /
    _finalize (one host thread per shard, two batches in flight); same JSON line as the multi-process
    path, plus the host time per batch of the caller and of the busiest shard thread."""
    _protect_stdout()
    import torch

    from hiprag import _native, synth

    n_vis = torch.cuda.device_count()
    devs = [i % max(1, n_vis) for i in range(args.gpus)]
    N, D, B, K = args.rows, args.dim, args.batch, args.k
    torch.cuda.set_device(devs[0])
    dev = torch.device("cuda", devs[0])
    t0 = time.time()
    index = _native.NativeIndex(D, args.dtype, "cosine", devices=devs)
    index.reserve(N)
    index.add_synthetic(args.seed, 0, N)
    torch.cuda.synchronize()
    log(f"one handle over devices {devs}: {N} rows built in {time.time() - t0:.1f}s")
    n_batches = args.warmup + args.steps
    q_dev = torch.from_numpy(np.stack([synth.planted_queries(args.seed, N, D, B, qseed=1000 + i)[0]
                                       for i in range(n_batches)])).to(dev)
    s_dev = torch.empty((n_batches, B, K), dtype=torch.float32, device=dev)
    r_dev = torch.empty((n_batches, B, K), dtype=torch.int64, device=dev)
    st = torch.cuda.current_stream(dev).cuda_stream

    # pipelined: submit enqueues batch i on every shard (one host thread per shard) and returns; the
    # handle keeps two batches in flight and finalizes the older one (guard flags, rare fallback) when a
    # third arrives; every batch is final before the clock stops
    def run(lo, hi):
        tickets = [index.search_submit(q_dev[i].data_ptr(), B, K, s_dev[i].data_ptr(), r_dev[i].data_ptr(), stream=st)
                   for i in range(lo, hi)]
        for t in tickets:
            index.search_finalize(t)

    run(0, args.warmup)
    for d in set(devs):
        torch.cuda.synchronize(d)
    h0 = index.host_us()
    t_start = time.perf_counter()
    run(args.warmup, n_batches)
    for d in set(devs):
        torch.cuda.synchronize(d)
    elapsed = time.perf_counter() - t_start
    h1 = index.host_us()
    nb = max(1, h1["batches"] - h0["batches"])
    host = {"caller_submit_us": round((h1["submit_us"] * h1["batches"] - h0["submit_us"] * h0["batches"]) / nb, 1),
            "busiest_shard_thread_us": round((h1["shard_thread_us"] * h1["batches"]
                                              - h0["shard_thread_us"] * h0["batches"]) / nb, 1)} if len(devs) > 1 else None
    result = {"metric": METRIC, "value": round(args.steps * B / elapsed, 2), "unit": "queries/s",
              "n_gpus": len(set(devs)), "steps": args.steps, "warmup": args.warmup,
              "ms_per_step": round(1000.0 * elapsed / args.steps, 4), "higher_is_better": True, "scaling": "strong",
              "vs_baseline": None, "dtype": args.dtype,
              "data": "synthetic: counter-based corpus generator (hiprag.synth), planted queries",
              "config": {"workload": f"{N / 1e6:g}M x {D} {args.dtype} cosine exact top-{K}, batch {B}, one handle "
                                     f"striped over {len(devs)} shards", "rows": N, "dim": D, "batch": B, "k": K,
                         "parallelism": f"onehandle{len(devs)}", "devices": devs},
              "host_us_per_batch": host}
    if not args.no_cpu:
        q_iso = isotropic_queries(B, D)
        qi_dev = torch.from_numpy(q_iso).to(dev)
        s_iso = torch.empty((B, K), dtype=torch.float32, device=dev)
        r_iso = torch.empty((B, K), dtype=torch.int64, device=dev)
        index.search_device(qi_dev.data_ptr(), B, K, s_iso.data_ptr(), r_iso.data_ptr(), stream=st)
        torch.cuda.synchronize(dev)
        nq = min(args.recall_queries, B)
        result.update(recall_checks(args, N, D, K, q_dev[args.warmup, :nq].cpu().numpy(),
                                    r_dev[args.warmup, :nq].cpu().numpy(), s_dev[args.warmup, :nq].cpu().numpy(),
                                    q_iso[:nq], r_iso[:nq].cpu().numpy(), s_iso[:nq].cpu().numpy()))
    emit(result)


def _free_port() -> int:
    import socket

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(args, argv) -> int:
    """``python bench.py --gpus N`` (N > 1) started without a torch.distributed launcher: start the N
    rank processes (torch.distributed.run, one rank per GPU, rendezvous on 127.0.0.1) as CHILDREN of
    this process and return their exit code.  This process never touches the GPU (no HIP call, no
    exec), so the ranks own the devices; rank 0's JSON line reaches stdout through the child."""
    import subprocess

    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__), *argv]
    log(f"launching {args.gpus} ranks: {' '.join(cmd[1:])}")
    return subprocess.run(cmd, env={**os.environ, "HIPRAG_BENCH_LAUNCHED": "1"}).returncode


def rank_env(args) -> tuple[int, int, int]:
    """(world, rank, local_rank) of this process; exits non-zero when the launcher's world size is
    not --gpus (a mismatch would otherwise print a line for the wrong number of GPUs)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"error: --gpus {args.gpus} but the launcher started WORLD_SIZE={world} ranks")
        sys.exit(2)
    return world, rank, local


def launch_probe(args) -> None:
    """--launch-probe (tests): the rank flow up to the process group, no GPU -- every rank joins a gloo
    group, rank 0 prints the world size the collective library sees and the ranks that answered."""
    import torch
    import torch.distributed as dist

    world, rank, _ = rank_env(args)
    if world > 1:
        dist.init_process_group("gloo")
    t = torch.ones(1)
    if world > 1:
        dist.all_reduce(t)
    if rank == 0:
        print(json.dumps({"n_gpus": dist.get_world_size() if world > 1 else 1, "ranks_answered": int(t.item()),
                          "launched_by_bench": os.environ.get("HIPRAG_BENCH_LAUNCHED") == "1"}), flush=True)
    if world > 1:
        dist.destroy_process_group()


_RESULT_OUT = None  # the process's original stdout (fd 1 goes to stderr while the GPU libraries run)


def _protect_stdout():
    """Keep stdout to the ONE JSON line: RCCL prints its version banner to fd 1 when a communicator comes up
    ("RCCL version : ...", seen in the --collective runs), and so may other libraries.  Fd 1 is pointed at
    stderr for the rest of the process and the result line goes to a duplicate of the original stdout."""
    global _RESULT_OUT
    if _RESULT_OUT is None:
        sys.stdout.flush()
        _RESULT_OUT = os.fdopen(os.dup(1), "w")
        os.dup2(2, 1)


def emit(result: dict) -> None:
    print(json.dumps(result), file=_RESULT_OUT or sys.stdout, flush=True)


def main():
    args = parse()
    if args.single_process:
        return main_single_process(args)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args, sys.argv[1:]))
    if args.launch_probe:
        return launch_probe(args)
    _protect_stdout()
    import torch
    import torch.distributed as dist

    from hiprag import _native, synth
    from hiprag.dist import ShardedSearch

    world, rank, local = rank_env(args)
    # rehearsal of the N > 1 flow on a one-GPU box (never the measured configuration): every rank on
    # GPU 0 and the gloo backend, as HIPRAG_BENCH_REHEARSE=1 (the exchange then takes the host path)
    rehearse = os.environ.get("HIPRAG_BENCH_REHEARSE") == "1"
    if rehearse:
        local = 0
    n_vis = torch.cuda.device_count()
    if local >= n_vis:
        log(f"error: rank {rank} needs GPU {local} but {n_vis} are visible (--gpus {args.gpus})")
        sys.exit(3)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        if rehearse:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=dev)
    elif args.collective:  # world size 1 through RCCL (no launcher: a private rendezvous on 127.0.0.1)
        dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0, world_size=1,
                                device_id=dev)
    # the rank count the collective library actually sees goes into the JSON line
    G = dist.get_world_size() if dist.is_initialized() else 1

    N, D, B, K = args.rows, args.dim, args.batch, args.k
    start = N * rank // G
    stop = N * (rank + 1) // G
    n_local = stop - start

    t0 = time.time()
    index = _native.NativeIndex(D, args.dtype, "cosine", device=local)
    index.set_persist(args.persist)
    index.set_q256(bool(args.q256))
    index.reserve(n_local)
    index.add_synthetic(args.seed, start, n_local)
    torch.cuda.synchronize()
    log(f"[rank {rank}] shard rows [{start}, {stop}) built in {time.time() - t0:.1f}s")

    # all query batches resident in HBM up front (planted queries: realistic margins)
    n_batches = args.warmup + args.steps
    qs = []
    for i in range(n_batches):
        q, _ = synth.planted_queries(args.seed, N, D, B, qseed=1000 + i)
        qs.append(q)
    q_dev = torch.from_numpy(np.stack(qs)).to(dev)
    q_ready = torch.cuda.Event()  # the queries are resident from here on (lets the search prep them early)
    q_ready.record()
    s_dev = torch.empty((n_batches, B, K), dtype=torch.float32, device=dev)
    r_dev = torch.empty((n_batches, B, K), dtype=torch.int64, device=dev)
    searcher = ShardedSearch(index, start, max_batch=B, device=dev, max_k=K, force_collective=args.collective,
                             depth=args.depth)

    # One step = one batch through the whole path.  Steps are pipelined two deep: submit()
    # enqueues batch i (scan, gather, merge, async copy of the guard flags) and finalizes the
    # batch submitted two steps earlier, so host work overlaps the GPU; every batch is fully
    # finalized (fallback included) before the clock stops.
    for i in range(args.warmup):
        searcher.submit(q_dev[i], K, s_out=s_dev[i], r_out=r_dev[i], q_ready=q_ready)
    searcher.finalize_all()
    torch.cuda.synchronize()
    index.take_scan_times()  # drop warmup launches
    # HIP events around every 8th SAMPLE+FILTER pair of the timed region (starting with the first;
    # three records: before SAMPLE, between the two, after FILTER): each event record leaves a
    # ~6 us bubble on the scan stream, so timing every launch would slow the steps being measured
    index.set_scan_timing(TIME_EVERY)
    wide0, q2560 = index.wide_launches(), index.q256_launches()
    persist0 = index.persist_stats()["batches"]
    fb0 = searcher.fallback_queries
    wait0 = searcher.wait_s
    if G > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t_start = time.perf_counter()
    for i in range(args.warmup, n_batches):
        searcher.submit(q_dev[i], K, s_out=s_dev[i], r_out=r_dev[i], q_ready=q_ready)
    searcher.finalize_all()
    torch.cuda.synchronize()
    if G > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t_start
    sample_ms, scan_ms = index.take_scan_times()
    wide_per_step = (index.wide_launches() - wide0) / args.steps  # 128-query FILTER launches per batch
    q256_per_step = (index.q256_launches() - q2560) / args.steps  # 256-query FILTER launches per batch
    pst = index.persist_stats()
    if pst["error"]:
        raise RuntimeError(f"persistent FILTER error {pst['error']}")
    persist = pst["batches"] - persist0 == args.steps  # every timed batch went through the persistent FILTER
    fallback_queries = searcher.fallback_queries - fb0  # guard failures in the timed region (collect fallback)
    host_wait_s = searcher.wait_s - wait0  # blocked on guard flags; the rest of the loop's wall time is host work
    persist_timeline = None
    if persist:  # where the period goes (device stamps, us): medians over the timed batches
        tr = index.persist_trace(args.steps)
        if len(tr) > 2:
            post, s0, s1, e0, e1 = (tr[:, j] for j in range(5))
            med = lambda x: round(float(np.median(x)), 2)  # noqa: E731
            persist_timeline = {
                "period_us": med(np.diff(e1)), "busy_us": med(e1 - s0),
                "start_spread_us": med(s1 - s0), "end_spread_us": med(e1 - e0),
                "post_before_prev_end_us": med(e1[:-1] - post[1:]),
                "first_start_after_prev_first_end_us": med(s0[1:] - e0[:-1]),
                "instances_run": int(pst["runs"])}
    # one untimed batch of isotropic queries (the worst case for ranking: no planted neighbour), for the
    # recall checks; every rank takes part (the merge is collective)
    q_iso = isotropic_queries(B, D)
    s_iso, r_iso = searcher.search(torch.from_numpy(q_iso).to(dev), K)
    torch.cuda.synchronize()
    if G > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        sc = torch.tensor([float(np.mean(scan_ms)), float(np.mean(sample_ms))], dtype=torch.float64, device=dev)
        dist.all_reduce(sc, op=dist.ReduceOp.MAX)
        scan_avg, sample_avg = float(sc[0]), float(sc[1])
    else:
        scan_avg, sample_avg = float(np.mean(scan_ms)), float(np.mean(sample_ms))

    # Every rank merges the same gathered candidates, so every rank must hold the same answers: a SHA-256 of each
    # rank's timed results (and the isotropic batch) is all-gathered and compared -- the
    # 8-GPU run proves its own cross-rank agreement instead of checking rank 0 against the oracle alone
    ranks_agree, digest = results_agree(torch, dist, dev, G, (s_dev[args.warmup:], r_dev[args.warmup:], s_iso, r_iso))

    qps = args.steps * B / elapsed
    ms_per_step = 1000.0 * elapsed / args.steps
    # corpus bytes per element the FILTER must read: fp32 rows are scanned through their 16-bit shadow (the values
    # the fp32 kernels rounded every fragment to; the exact rescoring reads fp32 -- hr_internal.hpp rows16) unless
    # HIPRAG_F32_SHADOW=0
    f32_shadow = args.dtype == "f32" and os.environ.get("HIPRAG_F32_SHADOW", "1") != "0"
    esz = 2 if f32_shadow else {"bf16": 2, "f16": 2, "f32": 4}[args.dtype]
    n_max_local = -(-N // G)
    alg_bytes = n_max_local * D * esz  # corpus bytes one filter-scan launch must read (largest shard)
    # FILTER launches per batch (the timed events bracket them all): 65-128 queries are one launch of the 128-query
    # FILTER (hr_wide.hip), 129-256 two -- counted by the index (hr_index_wide_launches); otherwise one launch
    wide = wide_per_step > 0
    q256 = q256_per_step > 0
    passes = max(1, round(wide_per_step)) if wide else 1
    achieved = passes * alg_bytes / (scan_avg * 1e-3) / 1e9 if scan_avg > 0 else 0.0
    mfma_flops = 2 * 32 * -(-B // 32) * n_max_local * D  # padded query slots x rows x dims per FILTER launch
    mfma_tflops = mfma_flops / (scan_avg * 1e-3) / 1e12 if scan_avg > 0 else 0.0

    result = {
        "metric": METRIC,
        "value": round(qps, 2),
        "unit": "queries/s",
        "n_gpus": G,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": args.dtype,
        "data": "synthetic: counter-based corpus generator (hiprag.synth), planted queries q = x_j/|x_j| + 0.05·eps",
        "config": {"workload": f"{N / 1e6:g}M x {D} {args.dtype} cosine exact top-{K}, batch {B}, row-sharded",
                   "rows": N, "dim": D, "batch": B, "k": K,
                   "parallelism": f"rowshard{G}" + ("+rccl" if searcher.collective else ""),
                   "exchange": (f"all-gather of the candidate records: {searcher.transport}" if searcher.collective
                                else "none (one shard: local copy)")},
        # the ranks' merged answers (timed batches + the isotropic batch) hash identically on every rank
        "ranks_agree": ranks_agree, "result_sha256": digest,
        "rccl_ranks": searcher.rccl.G if searcher.rccl is not None else None,
        "roofline": {"bound": "hbm",
                     "kernel": ("k_filter_q256 (256-query FILTER: one pass for four 64-query groups)" if q256 else
                                "k_filter_wide8 (128-query FILTER)" if wide else
                                "k_scan_persist (persistent FILTER; per-batch time = period between the device stamps "
                                "of consecutive batches' last workgroup arrivals)" if persist else "k_scan_filter (FILTER pass)"),
                     "filter_launches_per_batch": passes, "achieved": round(achieved, 1),
                     "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                     "frac_of_measured_read_ceiling": round(achieved / HBM_READ_CEILING_GBS, 4),
                     "read_ceiling_source": "profiles/r02_stream_ceiling.jsonl", "traffic": None,
                     "bytes_per_launch": alg_bytes, "scan_bytes_per_element": esz,
                     **({"scan_rows": "16-bit shadow of the fp32 rows"} if f32_shadow else {}),
                     "avg_launch_ms": round(scan_avg / passes, 4),
                     "sample_pass_ms": round(sample_avg, 4), "guard_fallback_queries": fallback_queries},
        # host work per step (submit minus its waits for guard flags): at or above ms_per_step the step is host-bound
        "host_ms_per_step": round(1000.0 * (elapsed - host_wait_s) / args.steps, 4),
        **({"persist_timeline": persist_timeline} if persist_timeline else {}),
        # the Q·Xᵀ contraction of the same launch on the MFMA pipe (bf16 dense peak, MI355X_MICROARCH.md)
        "mfma": {"achieved": round(mfma_tflops, 1), "peak": MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
                 "frac": round(mfma_tflops / MFMA_PEAK_TFLOPS, 4), "flops_per_launch": mfma_flops},
    }

    # PMC traffic of the same workload from the committed rocprofv3 summary (tools/profile.sh +
    # tools/summarize_profile.py): FETCH_SIZE x 2 (gfx950 correction) x 1024, per FILTER launch
    import glob

    # the FILTER launch's workload is the rank's shard, so a profile of that shard size on one GPU
    # (tools/profile.sh <tag> --rows n) serves every G that cuts the corpus into such shards
    suffixes = [f"_{N / 1e6:g}Mx{D}_b{B}_summary.json" if G == 1 else f"_{N / 1e6:g}Mx{D}_b{B}_g{G}_summary.json"]
    if D == 1024:
        suffixes.append(f"_shard{n_max_local / 1e6:g}M_b{B}_summary.json")
    summaries = []
    for suffix in suffixes:
        summaries = sorted(glob.glob(os.path.join(REPO, "profiles", "r*" + suffix)), key=summary_order)
        if summaries:
            break
    if summaries and args.dtype == "bf16" and K == 10:
        with open(summaries[-1]) as f:
            prof = json.load(f)
        if prof.get("k_scan_filter_mfma_busy_frac") is not None:
            result["mfma"]["pmc_busy_frac"] = round(prof["k_scan_filter_mfma_busy_frac"], 4)
            result["mfma"]["pmc_source"] = os.path.relpath(summaries[-1], REPO)
        if prof.get("hbm_read_bytes_per_launch"):  # the 128-query FILTER's summary (B > 64)
            result["roofline"]["traffic"] = round(prof["hbm_read_bytes_per_launch"] / 1e9, 3)
            result["roofline"]["traffic_unit"] = "GB per FILTER launch (HBM read, PMC)"
            result["roofline"]["traffic_source"] = os.path.relpath(summaries[-1], REPO)
            result["roofline"]["profiled_avg_launch_ms"] = prof.get("filter_ms_avg")
            result["roofline"]["profiled_launch_period_ms"] = prof.get("filter_period_ms_median")
        if prof.get("k_scan_filter_hbm_read_bytes"):
            result["roofline"]["traffic"] = round(prof["k_scan_filter_hbm_read_bytes"] / 1e9, 3)
            result["roofline"]["traffic_unit"] = "GB per launch (HBM read, PMC)"
            result["roofline"]["traffic_source"] = os.path.relpath(summaries[-1], REPO)
            result["roofline"]["profiled_avg_launch_ms"] = round(prof["k_scan_filter_ms_avg"], 4)
            if prof.get("k_scan_filter_period_ms_median"):  # start-to-start of consecutive FILTER launches
                result["roofline"]["profiled_launch_period_ms"] = round(prof["k_scan_filter_period_ms_median"], 4)
            if (prof.get("profiled_run") or {}).get("ms_per_step"):  # the bench line of that profiled run
                result["roofline"]["profiled_run_ms_per_step"] = prof["profiled_run"]["ms_per_step"]
            if prof.get("k_scan_sample_fetch_bytes"):  # the SAMPLE pass beside it (L3 hits included)
                result["roofline"]["sample_traffic"] = round(prof["k_scan_sample_fetch_bytes"] / 1e9, 3)
            if prof.get("k_scan_filter_busy_ms_per_launch"):  # overlapping launches (dual FILTER streams)
                result["roofline"]["profiled_busy_ms_per_launch"] = round(prof["k_scan_filter_busy_ms_per_launch"], 4)

    # recall@10 against the oracle's exact answer over the full corpus (rank 0)
    if rank == 0 and not args.no_cpu:
        nq = min(args.recall_queries, B)
        result.update(recall_checks(args, N, D, K, qs[args.warmup][:nq], r_dev[args.warmup, :nq].cpu().numpy(),
                                    s_dev[args.warmup, :nq].cpu().numpy(), q_iso[:nq],
                                    r_iso[:nq].cpu().numpy(), s_iso[:nq].cpu().numpy()))

    # the reference's embed + search query path on the GPU (N = 1), beside cpu_baseline's CPU embed + search
    if rank == 0 and G == 1 and not args.no_cpu and not args.no_embed:
        try:
            result["gpu_embed_plus_search"] = gpu_embed_plus_search(args, searcher, dev, D, K, B)
        except Exception as e:  # report, never hide
            result["gpu_embed_plus_search"] = {"error": repr(e)}

    # CPU baselines, rank 0, N=1 only: the reference's search path on the host cores (cpu_baseline),
    # the reference's per-query loop and the CPU query embedding beside it, and the exact fp64 oracle
    # (the checker, cpu_oracle) -- each on a bounded sample, scaled to the full corpus
    if rank == 0 and G == 1 and not args.no_cpu:
        try:
            result["cpu_baseline"] = cpu_reference_baseline(args, qs[args.warmup:], N, D, K, B)
        except Exception as e:  # report, never hide
            result["cpu_baseline"] = {"value": None, "error": repr(e)}
        try:
            import oracle
            from oracle import ref_numpy as R

            S = min(args.cpu_sample_rows, N)
            threads = oracle.default_threads()
            stored = oracle.c_build_synthetic(args.seed, 0, S, D, args.dtype, "cosine", threads)
            dt, nb = 0.0, 0
            while nb < args.steps and (dt < args.cpu_seconds / 2 or nb == 0):
                qn = R.process_queries(qs[args.warmup + nb], "cosine")
                t1 = time.perf_counter()
                oracle.c_search(stored, args.dtype, qn, K, nthreads=threads)
                dt += time.perf_counter() - t1
                nb += 1
            result["cpu_oracle"] = {"value": round(nb * B / (dt * (N / S)), 4), "unit": "queries/s", "cores": threads,
                                    "sample": f"exact fp64 checker (hr_oracle.c, OpenMP) of {nb} batches x {B} queries "
                                              f"over {S} of the {N} rows ({dt:.2f}s), scaled by {N / S:.1f}x"}
            del stored
        except Exception as e:
            result["cpu_oracle"] = {"value": None, "error": repr(e)}

    if rank == 0:
        emit(result)
    searcher.close()  # (every rank: the direct RCCL communicator goes before the process group)
    if G > 1:
        dist.barrier()
    if dist.is_initialized():
        dist.destroy_process_group()
    if not ranks_agree:
        log(f"[rank {rank}] error: the ranks' merged results differ")
        sys.exit(4)


def results_agree(torch, dist, dev, G: int, tensors) -> tuple[bool, str]:
    """(every rank holds the same bytes, this rank's SHA-256 hex) over `tensors` (device tensors, read back once
    after the timed region).  The 32-byte digests are all-gathered over the process group (device tensors for
    RCCL, host tensors for gloo)."""
    import hashlib

    h = hashlib.sha256()
    for t in tensors:
        h.update(t.contiguous().cpu().numpy().tobytes())
    digest = h.hexdigest()
    if G <= 1 or not dist.is_initialized():
        return True, digest
    mine = torch.from_numpy(np.frombuffer(h.digest(), np.int64).copy())
    if dist.get_backend() == "nccl":
        mine = mine.to(dev)
    every = [torch.empty_like(mine) for _ in range(G)]
    dist.all_gather(every, mine)
    return all(torch.equal(e, every[0]) for e in every), digest


if __name__ == "__main__":
    main()

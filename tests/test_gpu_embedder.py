"""GPU: the in-process embedder (PyTorch-ROCm forward + K7 HIP pooling) and the GPU ingest slice.

* K7 (hr_pool_normalize) vs the torch restatement of mean_pooling + F.normalize
  (tests/embed_ref.py <- deploying-locally.mdx:75-79, :114-115) on ragged masks, every
  hidden dtype and instruction lengths 0 / inside / past the sequence.  Tolerance: 1e-5
  absolute on unit vectors (fp32 sums in a different order; the NorthStar score tolerance).
* TorchRocmEmbedder.encode == the reference encode on the same model/tokenizer, fp32 and bf16.
* split -> embed -> hr_index_add_device -> BatchedVectorRetriever: stored rows bit-equal to the
  oracle's quantisation of the embedder output, ids identical to the oracle search.
"""
import asyncio

import numpy as np
import pytest
import torch

import oracle
from embed_ref import ref_mean_pooling, ref_passages, ref_queries
from hiprag import _native
from hiprag.rag import BatchedVectorRetriever, ChunkingConfig, Document, HipVectorStore, RetrieverConfig, VectorStoreConfig
from hiprag.rag.ingest import GpuIngestor
from hiprag.rag.rocm_embedder import TorchRocmEmbedder
from oracle import ref_numpy as R

pytestmark = pytest.mark.gpu
ATOL = 1e-5
DEV = torch.device("cuda", 0)
TD = {"f32": torch.float32, "bf16": torch.bfloat16, "f16": torch.float16}


@pytest.mark.parametrize("dt", ["f32", "bf16", "f16"])
@pytest.mark.parametrize("n_instr", [0, 3, 19])
def test_k7_pool_normalize_matches_torch(dt, n_instr):
    g = torch.Generator(device="cpu").manual_seed(7)
    B, T, H = 6, 37, 1000
    hidden = torch.randn((B, T, H), generator=g).to(DEV, TD[dt])
    lens = torch.tensor([37, 20, 1, 25, 19, 36])
    mask = (torch.arange(T)[None, :] < lens[:, None]).to(torch.int32).to(DEV)
    out = torch.empty((B, H), dtype=torch.float32, device=DEV)
    _native.pool_normalize(hidden.data_ptr(), dt, mask.data_ptr(), B, T, H, n_instr, out.data_ptr(),
                           torch.cuda.current_stream().cuda_stream)
    m = mask.clone()
    m[:, :n_instr] = 0
    ref = torch.nn.functional.normalize(ref_mean_pooling(hidden, m), dim=-1)
    torch.cuda.synchronize()
    # rows whose every token is masked are 0/0 = NaN in the reference too
    torch.testing.assert_close(out, ref, rtol=0, atol=ATOL, equal_nan=True)
    assert torch.isnan(out).any(1).tolist() == (m.sum(1) == 0).tolist()
    # packed K7 (the unpadded embedder's): the same rows as an (N, H) matrix + offsets -- bit-identical to
    # the padded kernel (same sums in the same order; the padded one only adds exact zeros besides)
    keep = mask.bool()
    packed = hidden[keep].contiguous()
    cu = torch.tensor([0, *torch.cumsum(lens, 0).tolist()], dtype=torch.int32, device=DEV)
    out_p = torch.empty_like(out)
    _native.pool_normalize_packed(packed.data_ptr(), dt, cu.data_ptr(), B, H, n_instr, out_p.data_ptr(),
                                  torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert torch.equal(torch.nan_to_num(out_p, nan=7.0), torch.nan_to_num(out, nan=7.0))


@pytest.mark.parametrize("dtype", ["float32", "bfloat16"])
def test_embedder_matches_reference_encode(dtype):
    # the padded Hugging Face forward, as the reference server runs it (the unpadded bf16 forward is
    # checked against this one below)
    emb = TorchRocmEmbedder(preset="bge-base", dtype=dtype, batch_size=8, max_length=128, seed=3, unpadded=False)
    texts = [f"passage {i}: " + " ".join(f"w{(i * 7 + j) % 97}" for j in range(5 + 11 * i)) for i in range(8)]
    got = emb.encode_passages(texts)
    ref = ref_passages(emb, texts)
    assert got.shape == (8, 768) and got.dtype == torch.float32
    torch.testing.assert_close(got, ref.float(), rtol=0, atol=ATOL)
    qs = ["what is w3?", "tell me about passage five and w12 w40"]
    torch.testing.assert_close(emb.encode_queries(qs), ref_queries(emb, qs).float(), rtol=0, atol=ATOL)
    v = asyncio.run(emb.embed_query(qs[0]))
    np.testing.assert_allclose(v, ref_queries(emb, qs[:1])[0].float().cpu().numpy(), atol=ATOL, rtol=0)


def test_ingest_split_embed_add_query(tmp_path):
    emb = TorchRocmEmbedder(preset="tiny", batch_size=32, max_length=128, seed=1)
    cfg = VectorStoreConfig(backend="hip", collection_name="kb", persist_directory=str(tmp_path),
                            index_params={"dtype": "bf16", "persist": True})
    store = HipVectorStore(cfg)
    ing = GpuIngestor(store, emb, chunking=ChunkingConfig(chunk_size=200, chunk_overlap=20), summary_index=False)
    seen = []  # the exact device vectors handed to the index
    inner = emb.embed_texts_device
    emb.embed_texts_device = lambda texts: seen.append(inner(texts)) or seen[-1]
    rng = np.random.default_rng(0)
    words = [f"term{i}" for i in range(400)]
    docs = [Document(id=f"doc{d}", content=". ".join(" ".join(rng.choice(words, 12)) for _ in range(20 + d)),
                     metadata={"source": f"s{d % 3}"}) for d in range(25)]
    n = asyncio.run(ing.ingest(docs))
    assert n == asyncio.run(store.count()) > 300
    # the stored rows are exactly the oracle's bf16 quantisation of the embedder's vectors
    records = [r for r in map(store.record, range(len(store._records))) if r is not None]
    vecs = torch.cat(seen).cpu().numpy()
    assert len(vecs) == len(records)
    rows = np.array([store._id_to_row[r["id"]] for r in records])
    assert (rows == np.arange(len(rows))).all()
    stored = store._index.get_rows(rows)
    expect = R.process_rows(vecs, "cosine", "bf16")
    np.testing.assert_array_equal(stored, R.dequantize(expect, "bf16"))
    # retrieval through the reference retriever API == oracle search over the same vectors
    queries = [" ".join(rng.choice(words, 6)) for _ in range(12)]
    got = asyncio.run(BatchedVectorRetriever(store, emb, RetrieverConfig(top_k=10, similarity_threshold=0.0))
                      .batch_retrieve(queries, top_k=10))
    qv = emb.encode_queries(queries).cpu().numpy()
    order = np.argsort(rows)
    s_ref, r_ref = oracle.c_search(expect[order], "bf16", R.process_queries(qv, "cosine"), 10)
    ids_sorted = [records[i]["id"] for i in order]
    assert [[r.chunk.id for r in res] for res in got] == [[ids_sorted[j] for j in rr] for rr in r_ref]
    for res, sr in zip(got, s_ref):
        np.testing.assert_allclose([r.score for r in res], sr, atol=ATOL, rtol=0)
    # persisted once at the end of the bulk ingest; a fresh store serves the same rows
    store2 = HipVectorStore(cfg)
    assert asyncio.run(store2.count()) == n


@pytest.mark.parametrize("dt", ["f32", "bf16", "f16"])
@pytest.mark.parametrize("H", [100, 768, 1024, 4096])
def test_k8_add_layernorm_matches_torch(dt, H):
    """K8 (hr_add_layernorm) vs PyTorch's add + F.layer_norm: fp32 within 1e-5; bf16 / f16 within one
    unit in the last place of the dtype, and bit-identical for nearly every element (the statistics
    are fp32 sums in another order than torch's Welford)."""
    g = torch.Generator(device="cpu").manual_seed(H)
    x = (torch.randn((37, H), generator=g) * 3).to(DEV, TD[dt])
    r = torch.randn((37, H), generator=g).to(DEV, TD[dt])
    w = (1 + 0.1 * torch.randn(H, generator=g)).to(DEV, TD[dt])
    b = (0.1 * torch.randn(H, generator=g)).to(DEV, TD[dt])
    out = _native.add_layernorm(x, r, w, b, 1e-12)
    ref = torch.nn.functional.layer_norm(x + r, (H,), w, b, 1e-12)
    torch.cuda.synchronize()
    if dt == "f32":
        torch.testing.assert_close(out, ref, rtol=0, atol=1e-5)
    else:
        ulp = 2.0 ** (-7 if dt == "bf16" else -10)
        diff = (out.float() - ref.float()).abs()
        assert bool((diff <= ulp * ref.float().abs().clamp_min(1.0)).all())
        assert float((out == ref).float().mean()) > 0.99


@pytest.mark.parametrize("dtype,atol", [("float32", 1e-5), ("bfloat16", 2e-2)])
def test_fused_layernorm_embedder_matches_unfused(dtype, atol):
    """The embedder with K8 in every encoder layer vs the same seeded model with PyTorch's add +
    LayerNorm: fp32 to 1e-5; bf16 to the accumulated rounding of 12 layers."""
    texts = [f"passage {i}: " + " ".join(f"w{(i * 5 + j) % 89}" for j in range(3 + 9 * i)) for i in range(6)]
    fused = TorchRocmEmbedder(preset="bge-base", dtype=dtype, batch_size=8, max_length=128, seed=4, fused_layernorm=True)
    plain = TorchRocmEmbedder(preset="bge-base", dtype=dtype, batch_size=8, max_length=128, seed=4, fused_layernorm=False)
    # 24 add+LayerNorm blocks (K8), and for the half model also its 12 exact-GELU intermediate blocks (hr_gelu_erf)
    assert fused.fused_layers == (24 if dtype == "float32" else 36) and plain.fused_layers == 0
    torch.testing.assert_close(fused.encode_passages(texts), plain.encode_passages(texts), rtol=0, atol=atol)


def test_ingest_writes_summary_vectors_that_kb_file_search_finds(tmp_path):
    """GpuIngestor adds each document's index_summary vector (processors.py:423-464), so the KB tools'
    kb_file_search (kb_search_toolkit.py:446-676) over a hiprag-built KB returns the files: every
    returned file's summary row is the exact top hit among the summary rows (oracle, same vectors)."""
    import json

    from hiprag.rag.kb_tools import KBSearchToolkit

    emb = TorchRocmEmbedder(preset="tiny", batch_size=64, max_length=96, seed=5)
    cfg = VectorStoreConfig(backend="hip", collection_name="kbsum", persist_directory=str(tmp_path),
                            index_params={"dtype": "bf16", "persist": False})
    store = HipVectorStore(cfg)
    seen = []
    inner = emb.embed_texts_device
    emb.embed_texts_device = lambda texts: seen.append(inner(texts)) or seen[-1]
    ing = GpuIngestor(store, emb, chunking=ChunkingConfig(chunk_size=150, chunk_overlap=10))
    rng = np.random.default_rng(4)
    words = [f"w{i}" for i in range(300)]
    docs = [Document(id=f"doc{d}", content=". ".join(" ".join(rng.choice(words, 8)) for _ in range(12)),
                     metadata={"source": f"file_{d}.pdf", "summary": " ".join(rng.choice(words, 10))})
            for d in range(30)]
    asyncio.run(ing.ingest(docs))
    recs = [store.record(i) for i in range(len(store._records))]
    summ_rows = [i for i, r in enumerate(recs) if r["metadata"].get("index_type") == "index_summary"]
    assert len(summ_rows) == 30 and all(recs[i]["id"].endswith("_summary") for i in summ_rows)
    tk = KBSearchToolkit(config={}, kb_resolver=lambda kb: ("kbsum", "kb"), store_factory=lambda c: store)
    tk._embedder_cache = emb
    out = json.loads(asyncio.run(tk.kb_file_search(kb_id=1, query=docs[7].metadata["summary"], top_k=5,
                                                   auto_rerank=False)))
    assert out["total_files"] == 5 and len(out["files"]) == 5
    vecs = torch.cat(seen).cpu().numpy()
    stored = R.process_rows(vecs, "cosine", "bf16")
    qv = R.process_queries(emb.encode_queries([docs[7].metadata["summary"]]).cpu().numpy(), "cosine")
    allowed = np.zeros(len(recs), bool)
    allowed[summ_rows] = True
    s_ref, r_ref = oracle.c_search(stored, "bf16", qv, 5, oracle.mask_from_bool(allowed))
    assert [f["file_name"] for f in out["files"]] == [recs[r]["metadata"]["source"] for r in r_ref[0]]


@pytest.mark.parametrize("dtype", ["bfloat16", "float16"])
def test_unpadded_embedder_matches_padded(dtype):
    """The encoder over the real tokens only (hiprag.rag.encoder: fused QKV GEMM, torch's varlen flash
    attention, no padded positions) vs Hugging Face's padded forward of the same seeded model: every
    pooled embedding within the half-precision rounding of 12 layers, cosine >= 0.999."""
    texts = [f"passage {i}: " + " ".join(f"w{(i * 11 + j) % 173}" for j in range(2 + 13 * (i % 9))) for i in range(40)]
    a = TorchRocmEmbedder(preset="bge-base", dtype=dtype, batch_size=16, max_length=256, seed=6)
    b = TorchRocmEmbedder(preset="bge-base", dtype=dtype, batch_size=16, max_length=256, seed=6, unpadded=False)
    assert a.unpadded is not None and a.unpadded.varlen is not None and b.unpadded is None
    x, y = a.encode_passages(texts), b.encode_passages(texts)
    torch.testing.assert_close(x, y, rtol=0, atol=2e-2)
    assert float((x * y).sum(1).min()) > 0.999
    torch.testing.assert_close(a.encode_queries(texts[:5]), b.encode_queries(texts[:5]), rtol=0, atol=2e-2)
    # several tokenizer batches per forward (forward_tokens): the same sequences through bigger GEMMs
    a.forward_tokens = 1000
    z = a.encode_passages(texts)
    torch.testing.assert_close(z, x, rtol=0, atol=2e-2)
    assert float((z * x).sum(1).min()) > 0.9999


@pytest.mark.parametrize("dtype", ["bfloat16", "float16"])
def test_graph_replayed_forward_matches_eager(dtype):
    """Query batches replayed from HIP graphs (encoder.GraphedForward: packed with a pad sequence up to a multiple
    of 64 tokens, the flash kernel's maximum length rounded up) vs the eager packed forward of the same model:
    every pooled embedding within half-precision rounding (the pad changes the GEMMs' row count, hence possibly
    their kernels), cosine >= 0.9999; batches of one shape reuse one graph; a forward above max_tokens runs
    eagerly."""
    texts = [f"query {i}: " + " ".join(f"w{(i * 7 + j) % 211}" for j in range(1 + 5 * (i % 7))) for i in range(96)]
    a = TorchRocmEmbedder(preset="bge-base", dtype=dtype, batch_size=32, max_length=256, seed=8)
    b = TorchRocmEmbedder(preset="bge-base", dtype=dtype, batch_size=32, max_length=256, seed=8, cuda_graphs=False)
    assert a.graphed is not None and b.graphed is None
    for lo in (0, 32, 64, 0, 32):  # three shapes, each seen twice
        x, y = a.encode_queries(texts[lo:lo + 32]), b.encode_queries(texts[lo:lo + 32])
        torch.testing.assert_close(x, y, rtol=0, atol=2e-2)
        assert float((x * y).sum(1).min()) > 0.9999
    assert a.graphed.replays == 5 and 1 <= len(a.graphed.graphs) <= 3
    a.graphed.max_tokens = 64  # every batch now exceeds it: eager
    n = a.graphed.replays
    torch.testing.assert_close(a.encode_queries(texts[:32]), b.encode_queries(texts[:32]), rtol=0, atol=2e-2)
    assert a.graphed.replays == n


@pytest.mark.parametrize("dtype", ["bfloat16", "float16"])
def test_short_attention_matches_sdpa(dtype):
    """hr_attn_varlen (one workgroup per sequence and head; S^T = K Q^T and O^T = V^T P^T on MFMA, fp32 softmax, P
    rounded to the input type as the flash kernel does) vs scaled_dot_product_attention of each sequence in fp32 on
    the same half-precision projections: within the rounding of P and of the output (2 ulps of the output type
    relative, plus an absolute floor).  Lengths 1..64 (a graph pack's pad sequence included), 70 sequences, 16 heads
    of 64; a sequence longer than 64 tokens is not its shape (None: the flash kernel's)."""
    import torch.nn.functional as F

    td = getattr(torch, dtype)
    g = torch.Generator(device="cpu").manual_seed(11)
    lengths = [1, 2, 7, 29, 31, 32, 33, 63, 64] + [int(x) for x in torch.randint(1, 60, (61,), generator=g)]
    nH, d = 16, 64
    cu_h = np.concatenate([[0], np.cumsum(lengths)]).astype(np.int64)
    n = int(cu_h[-1])
    qkv = (torch.randn((n, 3 * nH * d), generator=g) * 2.0).to(DEV, td)
    cu = torch.from_numpy(cu_h.astype(np.int32)).to(DEV)
    scale = d ** -0.5
    out = _native.attn_varlen(qkv, cu, len(lengths), nH, d, max(lengths), scale)
    assert out is not None and out.shape == (n, nH * d) and out.dtype == td
    x = qkv.float().view(n, 3, nH, d)
    ref = torch.empty((n, nH, d), dtype=torch.float32, device=DEV)
    for s, e in zip(cu_h[:-1], cu_h[1:]):
        qs, ks, vs = (x[s:e, i].transpose(0, 1) for i in range(3))
        ref[s:e] = F.scaled_dot_product_attention(qs, ks, vs, scale=scale).transpose(0, 1)
    ref = ref.reshape(n, nH * d)
    ulp = 2.0 ** (-8 if dtype == "bfloat16" else -11)
    err = (out.float() - ref).abs()
    floor = ulp * float(ref.abs().max())  # (P rounded to the input type: an absolute error of order ulp * max |v|)
    assert bool((err <= 2 * ulp * ref.abs() + floor).all()), float(err.max())
    assert float((out == ref.to(td)).float().mean()) > 0.5
    assert _native.attn_varlen(qkv, cu, len(lengths), nH, d, 65, scale) is None


@pytest.mark.parametrize("dtype", ["bfloat16", "float16"])
def test_gelu_erf_matches_torch(dtype):
    """hr_gelu_erf in place vs torch.nn.functional.gelu (approximate='none') on the same half-precision tensor:
    bf16 bit-identical (the same fp32 formula, rounded once); f16, whose 3 more bits expose last-bit differences of
    the fp32 intermediate, within one f16 ulp and identical on >= 99.9 % of the elements; a length that is not a
    multiple of 8 takes the tail path."""
    td = getattr(torch, dtype)
    g = torch.Generator(device="cpu").manual_seed(12)
    for n in (1, 13, 4096 * 1856, 1_000_003):
        x = (torch.randn(n, generator=g) * 3.0).to(DEV, td)
        want = torch.nn.functional.gelu(x)
        got = x.clone()
        assert _native.gelu_erf_(got) is got
        if dtype == "bfloat16":
            assert torch.equal(got, want), (n, float((got.float() - want.float()).abs().max()))
            continue
        diff = (got.float() - want.float()).abs()
        ulp = torch.where(want.float().abs() < 2.0 ** -14, torch.full_like(diff, 2.0 ** -24),
                          2.0 ** (torch.floor(torch.log2(want.float().abs().clamp_min(2.0 ** -14))) - 10))
        bad = diff > ulp
        if n > 1000:
            i = torch.nonzero(got != want)[:4, 0]
            print("f16 gelu differs at", x[i].tolist(), "ours", got[i].tolist(), "torch", want[i].tolist(),
                  "torch fp32", torch.nn.functional.gelu(x[i].float()).tolist())
        assert not bool(bad.any()), float(diff.max())
        assert float((got == want).float().mean()) >= 0.999

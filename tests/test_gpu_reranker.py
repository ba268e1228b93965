"""GPU: hr_topk_records against numpy, and the in-process cross-encoder reranker on the MI355X
(scores within 1e-5 of a torch fp32 pair-by-pair reference; per-query order = the kernel's (score
desc, position asc) selection; batched == per-query; retriever integration)."""
import asyncio

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _ref_topk(scores, ids, m):
    valid = ids >= 0
    s, r = scores[valid], ids[valid]
    order = np.lexsort((r, -s))[:m]
    out_s = np.full(m, -np.inf)
    out_r = np.full(m, -1, np.int64)
    out_s[:len(order)] = s[order]
    out_r[:len(order)] = r[order]
    return out_s, out_r


@pytest.mark.parametrize("m", [1, 10, 100, 1000])
def test_topk_records_vs_numpy(m):
    import torch

    from hiprag import _native

    rng = np.random.default_rng(m)
    lens = [0, 1, 5, 999, 1000, 1001, 4096, 70000]
    offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    n = int(offs[-1])
    scores = np.round(rng.standard_normal(n), 2)  # many exact ties
    ids = rng.permutation(n).astype(np.int64)
    ids[rng.random(n) < 0.05] = -1  # absent records
    rec = np.empty((n, 2), np.float64)
    rec[:, 0] = scores
    rec.view(np.int64)[:, 1] = ids
    rd = torch.from_numpy(rec).cuda()
    out = torch.empty((len(lens), m, 2), dtype=torch.float64, device="cuda")
    seg = torch.from_numpy(offs).cuda()
    _native.topk_records(rd.data_ptr(), len(lens), m, out.data_ptr(), seg_off_ptr=seg.data_ptr())
    torch.cuda.synchronize()
    got = out.cpu().numpy()
    for b in range(len(lens)):
        s_ref, r_ref = _ref_topk(scores[offs[b]:offs[b + 1]], ids[offs[b]:offs[b + 1]], m)
        np.testing.assert_array_equal(got[b].view(np.int64)[:, 1], r_ref)
        np.testing.assert_array_equal(got[b][:, 0], s_ref)


def test_reranker_scores_order_and_retriever():
    import torch

    from hiprag.rag import BatchedVectorRetriever, Chunk, RetrievalResult, RetrieverConfig
    from hiprag.rag.rerankers import TorchRocmReranker

    rr = TorchRocmReranker(preset="tiny", dtype="float32", batch_size=7, max_length=64)
    words = [f"w{i}" for i in range(300)]
    rng = np.random.default_rng(0)
    texts = [" ".join(rng.choice(words, rng.integers(1, 80))) for _ in range(60)]
    results = [RetrievalResult(chunk=Chunk(id=f"c{i}", document_id="d", content=t, chunk_index=i), score=0.1, rank=i + 1)
               for i, t in enumerate(texts)]
    query = "w1 w2 w3 w17"
    s = rr.score_pairs([query], [texts])[0].cpu().numpy()
    q_ids = rr._text_ids(query, cache=False)
    ref = []
    with torch.inference_mode():
        for t in texts:
            ids, types = rr._pair(q_ids, rr._text_ids(t, cache=True))
            logit = rr.model(input_ids=torch.tensor([ids], device="cuda"),
                             token_type_ids=torch.tensor([types], device="cuda")).logits[0, 0]
            ref.append(torch.sigmoid(logit.float()).item())
    np.testing.assert_allclose(s, ref, rtol=0, atol=1e-5)
    out = asyncio.run(rr.rerank(query, results, top_k=15))
    order = np.lexsort((np.arange(len(s)), -s.astype(np.float64)))[:15]
    assert [r.chunk.id for r in out] == [f"c{i}" for i in order]
    assert [r.rank for r in out] == list(range(1, 16))
    batch = rr.rerank_batch([query, "w5"], [results, results[:10]], top_k=15)
    assert [r.chunk.id for r in batch[0]] == [r.chunk.id for r in out] and len(batch[1]) == 10

    # through the retriever: 2*top_k candidates from the store, reranked to top_k (base_retriever.py:61-80)
    class Store:
        def search_batch(self, qvs, k, filters=None):
            return [[(r.chunk, 0.9 - 0.01 * i) for i, r in enumerate(results[:k])] for _ in qvs]

    class Emb:
        async def embed_query(self, q):
            return [0.0]

    ret = BatchedVectorRetriever(Store(), Emb(), RetrieverConfig(top_k=5, similarity_threshold=0.0), reranker=rr)
    got = asyncio.run(ret.batch_retrieve([query], top_k=5))[0]
    want = asyncio.run(rr.rerank(query, results[:10], top_k=5))
    assert [r.chunk.id for r in got] == [r.chunk.id for r in want]


def test_fused_layernorm_reranker_matches_unfused():
    """Cross-encoder scores with K8 in every XLM-R encoder layer vs PyTorch's add + LayerNorm (fp32)."""
    from hiprag.rag.rerankers import TorchRocmReranker

    words = [f"w{i}" for i in range(200)]
    rng = np.random.default_rng(3)
    texts = [" ".join(rng.choice(words, rng.integers(1, 60))) for _ in range(40)]
    a = TorchRocmReranker(preset="tiny", dtype="float32", batch_size=16, max_length=64, seed=2, fused_layernorm=True)
    b = TorchRocmReranker(preset="tiny", dtype="float32", batch_size=16, max_length=64, seed=2, fused_layernorm=False)
    assert a.fused_layers > 0 and b.fused_layers == 0
    np.testing.assert_allclose(a.score_pairs(["w1 w2 w9"], [texts])[0].cpu().numpy(),
                               b.score_pairs(["w1 w2 w9"], [texts])[0].cpu().numpy(), rtol=0, atol=1e-5)


def test_reranker_matches_hf_cross_encoder_fp32(golden_dir):
    """A local checkpoint (tests/golden/tiny_ce) scored by TorchRocmReranker on the GPU vs Hugging Face's own
    pair encoding (tokenizer(query, passage, truncation=True)) and forward on the CPU in fp32: relevance =
    sigmoid(logit) within 1e-5 for every pair, including truncated, empty and [UNK]-heavy passages."""
    import os

    import torch
    from transformers import AutoModelForSequenceClassification, AutoTokenizer

    from hiprag.rag.rerankers import TorchRocmReranker

    path = os.path.join(golden_dir, "tiny_ce")
    rr = TorchRocmReranker(path, dtype="float32", batch_size=5, max_length=64)
    tok = AutoTokenizer.from_pretrained(path, local_files_only=True)
    ref_model = AutoModelForSequenceClassification.from_pretrained(path, local_files_only=True).eval()
    words = open(os.path.join(path, "vocab.txt")).read().split()[13:]
    rng = np.random.default_rng(4)
    queries = ["which course grade", "revenue by region in the quarter?"]
    passages = [[" ".join(rng.choice(words, int(n))) for n in rng.integers(1, 90, 23)] + ["", "zyx qwv unknown"]
                for _ in queries]
    got = [s.cpu().numpy() for s in rr.score_pairs(queries, passages)]
    with torch.inference_mode():
        for q, ps, g in zip(queries, passages, got):
            # one call per pair: Hugging Face encodes text_pair="" as a single sequence only there
            want = [torch.sigmoid(ref_model(**tok(q, p, truncation=True, max_length=64, return_tensors="pt"))
                                  .logits[0, 0]).item() for p in ps]
            np.testing.assert_allclose(g, np.asarray(want, np.float32), rtol=0, atol=1e-5)


def test_unpadded_reranker_matches_padded_bf16():
    """Cross-encoder relevance through the unpadded encoder (varlen flash attention, fused QKV) vs the
    padded Hugging Face forward of the same seeded bf16 model."""
    from hiprag.rag.rerankers import TorchRocmReranker

    words = [f"w{i}" for i in range(200)]
    rng = np.random.default_rng(8)
    texts = [" ".join(rng.choice(words, rng.integers(1, 120))) for _ in range(70)]
    a = TorchRocmReranker(preset="bge-reranker-base", dtype="bfloat16", batch_size=32, max_length=256, seed=2)
    b = TorchRocmReranker(preset="bge-reranker-base", dtype="bfloat16", batch_size=32, max_length=256, seed=2,
                          unpadded=False)
    assert a.unpadded is not None and b.unpadded is None
    sa = a.score_pairs(["w1 w2 w9", "w5"], [texts, texts[:9]])
    sb = b.score_pairs(["w1 w2 w9", "w5"], [texts, texts[:9]])
    for x, y in zip(sa, sb):
        np.testing.assert_allclose(x.cpu().numpy(), y.cpu().numpy(), rtol=0, atol=2e-2)

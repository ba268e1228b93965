"""CPU tests of the in-process reranker's host logic (hiprag.rag.rerankers): the pair layout and
longest_first truncation against Hugging Face's own pair preparation, length-sorted batching that
scatters scores back to the right pairs, the reference's rerank semantics (openai_reranker.py
:83-121) and the factory.  The per-query selection runs on the GPU (hr_topk_records); here it is
replaced by a numpy stand-in -- tests/test_gpu_reranker.py covers the kernel."""
import asyncio
import os

import numpy as np
import pytest
import torch

from hiprag.rag import Chunk, RetrievalResult
from hiprag.rag.rerankers import RerankerFactory, TorchRocmReranker, build_random_cross_encoder


def _numpy_select(self, scores, top_ns):
    out = []
    for s, n in zip(scores, top_ns):
        s = s.cpu().numpy().astype(np.float64)
        order = np.lexsort((np.arange(len(s)), -s))[: min(n, len(s))]
        out.append([(int(p), float(s[p])) for p in order])
    return out


@pytest.fixture
def cpu_reranker(monkeypatch):
    monkeypatch.setattr(TorchRocmReranker, "_select", _numpy_select)
    return TorchRocmReranker(preset="tiny", device="cpu", dtype="float32", batch_size=3, max_length=24)


def test_pair_layout_matches_huggingface(tmp_path):
    from transformers import BertTokenizer

    vocab = ["[PAD]", "[UNK]", "[CLS]", "[SEP]", "[MASK]"] + [f"w{i}" for i in range(50)]
    (tmp_path / "vocab.txt").write_text("\n".join(vocab))
    tok = BertTokenizer(str(tmp_path / "vocab.txt"))
    rng = np.random.default_rng(0)
    for _ in range(200):
        a = list(rng.integers(5, 55, rng.integers(0, 30)))
        b = list(rng.integers(5, 55, rng.integers(0, 60)))
        L = int(rng.integers(3, 70))
        ref = tok(" ".join(vocab[x] for x in a), " ".join(vocab[x] for x in b), truncation="longest_first",
                  max_length=L, add_special_tokens=True)
        rr = TorchRocmReranker.__new__(TorchRocmReranker)
        rr.tokenizer, rr.max_length = tok, L
        ids, types = rr._pair([int(x) for x in a], [int(x) for x in b], passage_is_empty=not b)
        assert ids == ref["input_ids"] and types == ref["token_type_ids"], (a, b, L)


def test_scores_scatter_back_and_match_single_pairs(cpu_reranker):
    rr = cpu_reranker
    queries = ["what is the capital of france", "gpu kernels"]
    passages = [["paris is the capital", "berlin", "a b c d e f g h i j k l m n o p q r s t u v w x y z"],
                ["hip kernels on mi355x", "", "kernels", "lds and hbm bandwidth of the gpu"]]
    got = rr.score_pairs(queries, passages)
    for q, ps, s in zip(queries, passages, got):
        q_ids = rr._text_ids(q, cache=False)
        for p, v in zip(ps, s.tolist()):
            ids, types = rr._pair(q_ids, rr._text_ids(p, cache=True), passage_is_empty=not p)
            with torch.inference_mode():
                logit = rr.model(input_ids=torch.tensor([ids]), token_type_ids=torch.tensor([types]),
                                 attention_mask=torch.ones(1, len(ids), dtype=torch.long)).logits[0, 0]
            assert abs(torch.sigmoid(logit).item() - v) < 1e-5
    assert "hip kernels on mi355x" in rr._cache  # passages cached, queries not
    assert queries[1] not in rr._cache


def _results(texts):
    return [RetrievalResult(chunk=Chunk(id=f"c{i}", document_id="d", content=t, chunk_index=i), score=0.5, rank=i + 1)
            for i, t in enumerate(texts)]


def test_rerank_semantics(cpu_reranker):
    rr = cpu_reranker
    res = _results(["alpha beta", "gamma", "alpha", "delta epsilon zeta", "beta"])
    assert asyncio.run(rr.rerank("q", [], top_k=3)) == []
    out = asyncio.run(rr.rerank("alpha", res, top_k=3))
    s = rr.score_pairs(["alpha"], [[r.chunk.content for r in res]])[0].numpy().astype(np.float64)
    order = np.lexsort((np.arange(5), -s))[:3]
    assert [r.chunk.id for r in out] == [f"c{i}" for i in order]
    assert [r.rank for r in out] == [1, 2, 3]
    np.testing.assert_allclose([r.score for r in out], s[order], rtol=0, atol=1e-7)
    assert len(asyncio.run(rr.rerank("alpha", res))) == 5  # top_k None -> all
    batch = rr.rerank_batch(["alpha", "gamma"], [res, res[:2]], top_k=2)
    assert [r.chunk.id for r in batch[0]] == [r.chunk.id for r in out[:2]]
    assert len(batch[1]) == 2


def test_rerank_failure_returns_retrieval_order(monkeypatch, cpu_reranker):
    def boom(*a, **k):
        raise RuntimeError("device lost")

    monkeypatch.setattr(cpu_reranker, "score_pairs", boom)
    res = _results(["a", "b", "c"])
    assert asyncio.run(cpu_reranker.rerank("q", res, top_k=2)) == res[:2]


def test_factory(monkeypatch):
    monkeypatch.delenv("UTU_RERANKER_URL", raising=False)
    with pytest.raises(ValueError):
        RerankerFactory.create("auto")
    with pytest.raises(ValueError):
        RerankerFactory.create("service")
    with pytest.raises(ValueError):
        RerankerFactory.create("milvus")
    with pytest.raises(NotImplementedError):
        RerankerFactory.create("jina", api_key="x")
    m = build_random_cross_encoder("tiny", seed=3)
    assert m.config.num_labels == 1 and m.config.hidden_size == 256


def test_vectorised_pair_batches_match_per_pair_forward():
    """score_pairs assembles length-sorted batches with numpy (query / passage / [SEP] scatter, token
    types, masks, longest_first truncation, empty passages as single sequences): on the CPU its scores
    equal a per-pair forward of rr._pair's encoding, for a max_length that truncates."""
    import numpy as np
    import torch

    from hiprag.rag.rerankers import TorchRocmReranker

    rr = TorchRocmReranker(preset="tiny", dtype="float32", batch_size=7, max_length=24, device="cpu")
    words = [f"w{i}" for i in range(300)]
    rng = np.random.default_rng(1)
    queries = ["w1 w2 w3", " ".join(rng.choice(words, 30)), "w9"]
    passages = [[" ".join(rng.choice(words, int(k))) for k in rng.integers(1, 40, 9)] + [""] for _ in queries]
    got = [s.numpy() for s in rr.score_pairs(queries, passages)]
    with torch.inference_mode():
        for q, ps, g in zip(queries, passages, got):
            q_ids = rr._text_ids(q, cache=False)
            want = []
            for p in ps:
                ids, types = rr._pair(q_ids, rr._text_ids(p, cache=True), passage_is_empty=not p)
                assert len(ids) <= 24
                logit = rr.model(input_ids=torch.tensor([ids]), token_type_ids=torch.tensor([types])).logits[0, 0]
                want.append(torch.sigmoid(logit.float()).item())
            np.testing.assert_allclose(g, want, rtol=0, atol=1e-5)

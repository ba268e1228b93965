"""Embedder parity against the REFERENCE server's own model code (tests/golden/gen_embedder.py ran the
LLMEmbeddingModel listing of deploying-locally.mdx:41-126 on the build container's CPU over the committed
tiny seeded BERT in tests/golden/tiny_bert/).

CPU: the torch restatement tests/embed_ref.py (the K7 numerics oracle) reproduces the fixture -- the
oracle is pinned by the reference itself.  GPU: hiprag's TorchRocmEmbedder (PyTorch-ROCm forward + the K7
HIP pooling kernel) reproduces it within 1e-5 (fp32 model)."""
import json
import os
import types

import numpy as np
import pytest
import torch

from embed_ref import ref_passages, ref_queries


@pytest.fixture(scope="module")
def golden(golden_dir):
    meta = json.load(open(os.path.join(golden_dir, "embedder_golden.json")))
    meta["emb"] = np.load(os.path.join(golden_dir, "embedder_golden.npy"))
    meta["path"] = os.path.join(golden_dir, meta["model_dir"])
    return meta


def _split(golden, out):
    nq = len(golden["queries"])
    return out[:nq], out[nq:]


def test_restatement_matches_reference_listing(golden):
    from transformers import AutoModel, AutoTokenizer

    model = AutoModel.from_pretrained(golden["path"], local_files_only=True).eval()
    tok = AutoTokenizer.from_pretrained(golden["path"], padding_side="right", local_files_only=True)
    emb = types.SimpleNamespace(model=model, tokenizer=tok, max_length=golden["max_length"], device=torch.device("cpu"),
                                query_instruction=golden["query_instruction"], doc_instruction=golden["doc_instruction"])
    q = ref_queries(emb, golden["queries"]).numpy()
    p = ref_passages(emb, golden["passages"]).numpy()
    gq, gp = _split(golden, golden["emb"])
    np.testing.assert_allclose(q, gq, atol=1e-6, rtol=0)
    np.testing.assert_allclose(p, gp, atol=1e-6, rtol=0)


@pytest.mark.gpu
def test_rocm_embedder_matches_reference_listing(golden):
    from hiprag.rag.rocm_embedder import TorchRocmEmbedder

    emb = TorchRocmEmbedder(golden["path"], dtype="float32", max_length=golden["max_length"], batch_size=128)
    assert emb.fused_layers > 0  # the K8 fused add+LayerNorm path is the one under test
    q = emb.encode_queries(golden["queries"]).cpu().numpy()
    p = emb.encode_passages(golden["passages"]).cpu().numpy()
    gq, gp = _split(golden, golden["emb"])
    np.testing.assert_allclose(q, gq, atol=1e-5, rtol=0)
    np.testing.assert_allclose(p, gp, atol=1e-5, rtol=0)
    # the async BaseEmbedder API returns the same vectors as host lists
    import asyncio

    one = asyncio.run(emb.embed_query(golden["queries"][0]))
    np.testing.assert_allclose(np.asarray(one, np.float32), gq[0], atol=1e-5, rtol=0)

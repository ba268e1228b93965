"""CPU: the unpadded encoder forward (hiprag.rag.encoder) equals Hugging Face's padded forward at every
real token -- embedder (BertModel) and cross-encoder (BertForSequenceClassification logits) -- for
right-padded ragged batches, with the per-sequence SDPA attention (the varlen flash kernel that serves
fp16 / bf16 models on the GPU is checked in tests/test_gpu_embedder.py)."""
import numpy as np
import torch

from hiprag.rag.encoder import UnpaddedEncoder, sequence_logits
from hiprag.rag.rerankers import build_random_cross_encoder
from hiprag.rag.rocm_embedder import build_random_bert


def _batch(rng, B, T, vocab=30522):
    lens = rng.integers(3, T + 1, B)
    lens[0] = T
    ids = np.zeros((B, T), np.int64)
    for b, n in enumerate(lens):
        ids[b, :n] = rng.integers(1000, vocab, n)
        ids[b, 0], ids[b, n - 1] = 101, 102
    mask = (np.arange(T)[None, :] < lens[:, None]).astype(np.int64)
    return torch.from_numpy(ids), torch.from_numpy(mask), lens


def test_unpadded_encoder_matches_padded_forward():
    torch.manual_seed(0)
    model = build_random_bert("tiny", 3).eval()
    enc = UnpaddedEncoder(model, use_varlen=False)
    rng = np.random.default_rng(5)
    for B, T in ((1, 7), (5, 33), (9, 64)):
        ids, mask, lens = _batch(rng, B, T)
        with torch.inference_mode():
            ref = model(input_ids=ids, attention_mask=mask)[0]
            got = enc(ids, lens)
        keep = mask.bool()
        torch.testing.assert_close(got[keep], ref[keep], rtol=1e-5, atol=2e-5)
        assert torch.count_nonzero(got[~keep]) == 0


def test_unpadded_cross_encoder_logits_match():
    torch.manual_seed(0)
    model = build_random_cross_encoder("bge-reranker-base", 4, num_hidden_layers=2, hidden_size=128,
                                       num_attention_heads=4, intermediate_size=256).eval()
    enc = UnpaddedEncoder(model.base_model, use_varlen=False)
    assert sequence_logits(model, None, probe=True)
    rng = np.random.default_rng(6)
    ids, mask, lens = _batch(rng, 7, 40)
    types = torch.from_numpy((np.arange(40)[None, :] >= (lens // 2)[:, None]).astype(np.int64)) * mask
    with torch.inference_mode():
        ref = model(input_ids=ids, attention_mask=mask, token_type_ids=types).logits
        got = sequence_logits(model, enc(ids, lens, types))
    torch.testing.assert_close(got, ref, rtol=1e-5, atol=2e-5)


def test_packed_forward_matches_padded_bert_and_xlmr():
    """pack() + forward_packed(): every packed row equals the padded forward's row of that token, for
    BERT (absolute positions 0..L-1) and XLM-R (positions padding_idx + 1 + t) embeddings."""
    from transformers import XLMRobertaConfig, XLMRobertaModel

    torch.manual_seed(0)
    xlmr = XLMRobertaModel(XLMRobertaConfig(vocab_size=2000, hidden_size=64, num_hidden_layers=2,
                                            num_attention_heads=4, intermediate_size=128, pad_token_id=1,
                                            max_position_embeddings=80), add_pooling_layer=False).eval()
    rng = np.random.default_rng(8)
    for model, vocab in ((build_random_bert("tiny", 3).eval(), 30522), (xlmr, 2000)):
        enc = UnpaddedEncoder(model, use_varlen=False)
        for B, T in ((1, 5), (6, 40)):
            ids, mask, lens = _batch(rng, B, T, vocab)
            if vocab == 2000:
                ids[~mask.bool()] = 1  # XLM-R pads with its padding_idx
            types = torch.zeros_like(ids)
            with torch.inference_mode():
                ref = model(input_ids=ids, attention_mask=mask, token_type_ids=types)[0]
                pk = enc.pack(ids, mask, types)
                got = enc.forward_packed(pk)
            assert pk.cu.dtype == torch.int32 and pk.cu.tolist() == [0, *np.cumsum(lens).tolist()]
            torch.testing.assert_close(got, ref[mask.bool()], rtol=1e-5, atol=2e-5)


def test_packed_cross_encoder_head_and_left_padding_refused():
    import pytest

    from hiprag.rag.encoder import first_tokens

    torch.manual_seed(0)
    model = build_random_cross_encoder("bge-reranker-base", 4, num_hidden_layers=2, hidden_size=128,
                                       num_attention_heads=4, intermediate_size=256).eval()
    enc = UnpaddedEncoder(model.base_model, use_varlen=False)
    rng = np.random.default_rng(9)
    ids, mask, lens = _batch(rng, 5, 30)
    types = torch.from_numpy((np.arange(30)[None, :] >= (lens // 2)[:, None]).astype(np.int64)) * mask
    with torch.inference_mode():
        ref = model(input_ids=ids, attention_mask=mask, token_type_ids=types).logits
        pk = enc.pack(ids.numpy(), mask.numpy(), types.numpy())
        got = sequence_logits(model, first_tokens(enc.forward_packed(pk), pk.cu_host))
    torch.testing.assert_close(got, ref, rtol=1e-5, atol=2e-5)
    with pytest.raises(ValueError):
        enc.pack(ids, mask.flip(1))


def test_pack_of_several_batches_is_their_concatenation():
    torch.manual_seed(0)
    model = build_random_bert("tiny", 3).eval()
    enc = UnpaddedEncoder(model, use_varlen=False)
    rng = np.random.default_rng(10)
    (i1, m1, l1), (i2, m2, l2) = _batch(rng, 3, 12), _batch(rng, 4, 30)
    with torch.inference_mode():
        both = enc.pack([i1, i2], [m1, m2])
        h = enc.forward_packed(both)
        a, b = enc.forward_packed(enc.pack(i1, m1)), enc.forward_packed(enc.pack(i2, m2))
    assert both.lengths.tolist() == [*l1.tolist(), *l2.tolist()] and both.max_len == 30
    torch.testing.assert_close(h, torch.cat([a, b]), rtol=1e-5, atol=2e-5)


def test_graphed_forward_only_captures_varlen_layers():
    """a captured forward must not bake in host-sliced attention.  graph_safe() holds only when every
    layer takes the varlen kernel (offsets read from the device tensor); GraphedForward runs everything else eagerly."""
    from hiprag.rag.encoder import GraphedForward

    torch.manual_seed(0)
    model = build_random_bert("tiny", 3).eval()
    enc = UnpaddedEncoder(model, use_varlen=False)
    assert not enc.graph_safe()  # SDPA per sequence, sliced by host offsets
    enc.varlen = lambda *a: None  # a varlen kernel: every layer's 1/sqrt(d) scale takes it
    assert enc.graph_safe()
    w, b, nH, d, scale, *rest = enc.layers[1]
    enc.layers[1] = (w, b, nH, d, scale * 2.0, *rest)  # one layer with its own scale falls back to SDPA
    assert not enc.graph_safe()
    enc = UnpaddedEncoder(model, use_varlen=False)
    g = GraphedForward(enc)
    rng = np.random.default_rng(7)
    ids, mask, lens = _batch(rng, 4, 16)
    with torch.inference_mode():
        pk = enc.pack(ids, mask, granule=16)
        out = g(pk)
    assert not g.graphs and g.replays == 0 and out.shape[0] == int(pk.cu_host[-1])

"""Unpadded (variable-length) forward of the BERT / XLM-R encoders behind the in-process embedder and
cross-encoder (PyTorch-ROCm: the one place the package computes with torch, BASELINE north_star).

Hugging Face's forward runs every encoder GEMM over the padded batch (B x T positions) and masks the
padding in attention.  Here the embeddings are computed on the padded batch (so position and token-type
ids are exactly Hugging Face's), then only the real tokens go through the layers, packed as one
(N, H) matrix:
  * Q, K and V come from ONE GEMM (the three projections' weights concatenated once, (3H, H));
  * attention is torch's variable-length flash attention over the packed tokens (cumulative sequence
    lengths; no mask, no padded keys), or, where it does not exist (CPU, fp32), plain SDPA per sequence;
  * the attention output and FFN blocks are the model's own modules (dense + residual + LayerNorm -- K8
    when fuse_encoder_layers patched them -- and the intermediate dense + activation), called on 2-D
    token matrices.
Every real position's output equals the padded forward's (the padded keys carry zero weight there);
padded positions come back as zeros, which the masked pooling (K7) and the CLS heads never read.
The per-sequence lengths are host values (the caller built the right-padded batch on the host), so no
device-to-host sync is needed for the packing indices or the flash kernel's maximum length.
"""
from __future__ import annotations

import os

import numpy as np

_ENV = os.environ.get("HIPRAG_UNPADDED", "1") != "0"  # A/B switch


def _varlen():
    try:
        from torch.nn.attention.varlen import varlen_attn
    except Exception:  # noqa: BLE001 -- older torch: no varlen flash attention
        return None
    return varlen_attn


def _sdpa_per_sequence(q, k, v, cu_host, max_len, scale):
    """Reference attention over packed tokens: SDPA on each sequence ((N, nH, d) -> (N, nH, d))."""
    import torch.nn.functional as F

    out = q.new_empty(q.shape)
    for s, e in zip(cu_host[:-1], cu_host[1:]):
        s, e = int(s), int(e)
        if e == s:
            continue
        qs, ks, vs = (x[s:e].transpose(0, 1) for x in (q, k, v))  # (nH, L, d)
        out[s:e] = F.scaled_dot_product_attention(qs, ks, vs, scale=scale).transpose(0, 1)
    return out


class UnpaddedEncoder:
    """The layers of `base_model` (a BertModel / XLMRobertaModel: .embeddings, .encoder.layer) over the
    real tokens of right-padded batches.  use_varlen: None = torch's flash varlen kernel when the model
    is fp16 / bf16 on a GPU, else SDPA per sequence."""

    def __init__(self, base_model, use_varlen: bool | None = None):
        import torch

        self.torch = torch
        self.emb = base_model.embeddings
        self.layers = []
        p = next(base_model.parameters())
        for layer in base_model.encoder.layer:
            sa = layer.attention.self
            w = torch.cat([sa.query.weight, sa.key.weight, sa.value.weight]).contiguous()
            b = torch.cat([sa.query.bias, sa.key.bias, sa.value.bias]).contiguous()
            scale = float(getattr(sa, "scaling", sa.attention_head_size ** -0.5))
            self.layers.append((w, b, sa.num_attention_heads, sa.attention_head_size, scale,
                                layer.attention.output, layer.intermediate, layer.output))
        va = _varlen()
        if use_varlen is None:
            use_varlen = va is not None and p.is_cuda and p.dtype in (torch.float16, torch.bfloat16)
        if use_varlen and va is None:
            raise RuntimeError("torch.nn.attention.varlen is not available")
        self.varlen = va if use_varlen else None
        self.observers = []  # callables (B, T, lengths) per forward (tools/flops.py counts FLOPs with it)

    @staticmethod
    def supported(base_model) -> bool:
        layers = getattr(getattr(base_model, "encoder", None), "layer", None)
        if not layers or not hasattr(base_model, "embeddings"):
            return False
        sa = getattr(getattr(layers[0], "attention", None), "self", None)
        return all(hasattr(sa, n) for n in ("query", "key", "value", "num_attention_heads", "attention_head_size")) \
            and not getattr(getattr(base_model, "config", None), "is_decoder", False)

    def __call__(self, input_ids, lengths, token_type_ids=None):
        """input_ids (B, T) device, right-padded; lengths: host int array (B,) of real tokens per row.
        Returns the last hidden state (B, T, H) with zeros at padded positions."""
        torch = self.torch
        B, T = input_ids.shape
        dev = input_ids.device
        lengths = np.asarray(lengths, np.int64)
        cu = np.zeros(B + 1, np.int64)
        cu[1:] = np.cumsum(lengths)
        n = int(cu[-1])
        idx_h = (np.repeat(np.arange(B, dtype=np.int64) * T, lengths)
                 + np.arange(n, dtype=np.int64) - np.repeat(cu[:-1], lengths))
        pin = dev.type == "cuda"
        idx = torch.from_numpy(idx_h)
        cu_t = torch.from_numpy(cu.astype(np.int32))
        if pin:
            idx, cu_t = idx.pin_memory(), cu_t.pin_memory()
        idx, cu_t = idx.to(dev, non_blocking=pin), cu_t.to(dev, non_blocking=pin)
        max_len = int(lengths.max()) if B else 0
        for f in self.observers:
            f(B, T, lengths)
        x = self.emb(input_ids=input_ids, token_type_ids=token_type_ids)  # Hugging Face's positions / types
        H = x.shape[-1]
        h = x.reshape(B * T, H).index_select(0, idx)
        for w, b, nH, d, scale, attn_out, inter, out in self.layers:
            qkv = torch.nn.functional.linear(h, w, b).view(n, 3, nH, d)
            q, k, v = (qkv[:, i].contiguous() for i in range(3))
            if self.varlen is not None and abs(scale * d ** 0.5 - 1.0) < 1e-6:  # (the kernel's own 1/sqrt(d))
                a = self.varlen(q, k, v, cu_t, cu_t, max_len, max_len)
            else:
                a = _sdpa_per_sequence(q, k, v, cu, max_len, scale)
            h = attn_out(a.reshape(n, nH * d), h)
            h = out(inter(h), h)
        seq = x.new_zeros(B * T, H)
        seq.index_copy_(0, idx, h)
        return seq.view(B, T, H)


def sequence_logits(model, seq, probe: bool = False):
    """Classification logits of a *ForSequenceClassification model from its encoder's last hidden state
    (B, T, H): Bert (pooler on [CLS] -> dropout -> classifier) or RoBERTa / XLM-R (classifier head on the
    first token).  None for other heads (the caller then runs the model's own forward); probe=True only
    answers whether the head is one of these."""
    if probe:
        return (hasattr(model, "bert") or hasattr(model, "roberta")) and hasattr(model, "classifier")
    if hasattr(model, "bert") and hasattr(model, "classifier"):
        pooled = model.bert.pooler(seq) if model.bert.pooler is not None else seq[:, 0]
        return model.classifier(model.dropout(pooled))
    if hasattr(model, "roberta") and hasattr(model, "classifier"):
        return model.classifier(seq)
    return None

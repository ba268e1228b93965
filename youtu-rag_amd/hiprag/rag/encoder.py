"""Unpadded (variable-length) forward of the BERT / XLM-R encoders behind the in-process embedder and
cross-encoder (PyTorch-ROCm: the one place the package computes with torch, BASELINE north_star).

Hugging Face's forward runs every encoder GEMM over the padded batch (B x T positions) and masks the
padding in attention.  Here only the real tokens are computed, packed as one (N, H) matrix:
  * the embeddings are the model's own module over the packed ids, token types and Hugging Face's
    position ids of each token (0..L-1, or padding_idx + 1 + 0..L-1 for RoBERTa / XLM-R);
  * Q, K and V come from ONE GEMM (the three projections' weights concatenated once, (3H, H)) and go to
    the attention as strided views of its output;
  * attention is torch's variable-length flash attention over the packed tokens (cumulative sequence
    lengths; no mask, no padded keys), or, where it does not exist (CPU, fp32), plain SDPA per sequence;
  * the attention output and FFN blocks are the model's own modules (dense + residual + LayerNorm -- K8
    when fuse_encoder_layers patched them -- and the intermediate dense + activation), called on 2-D
    token matrices.
Every real position's output equals the padded forward's (the padded keys carry zero weight there).
pack() builds the packed batch on the host from the tokenizer's right-padded output and uploads it in
one pinned copy; the embedder pools it with the packed K7 (hr_pool_normalize_packed) and the
cross-encoder's head reads each sequence's first row.  __call__ keeps the padded (B, T, H) interface
(zeros at padded positions) for callers holding a device batch.  Lengths are host values throughout, so
no device-to-host sync is needed for the packing or the flash kernel's maximum length.
"""
from __future__ import annotations

import os
from typing import Any, NamedTuple

import numpy as np

_ENV = os.environ.get("HIPRAG_UNPADDED", "1") != "0"  # A/B switch
_SHORT = os.environ.get("HIPRAG_SHORT_ATTN", "1") != "0"  # A/B switch: hr_attn_varlen for short sequences


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
        self.device = next(base_model.parameters()).device
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
        # batches whose sequences are all at most 64 tokens (queries; the graph-replayed query forwards) take the
        # short-sequence attention kernel (hr_attn_varlen: one workgroup per sequence and head, S and P V on MFMA)
        # instead of the flash kernel, whose tiles are sized for long sequences (19 us + a 5 us fill per layer at
        # 64 queries)
        self.short_attn = _SHORT and p.is_cuda and p.dtype in (torch.float16, torch.bfloat16)
        self.observers = []  # callables (B, T, lengths) per forward (tools/flops.py counts FLOPs with it)

    @staticmethod
    def supported(base_model) -> bool:
        layers = getattr(getattr(base_model, "encoder", None), "layer", None)
        if not layers or not hasattr(base_model, "embeddings"):
            return False
        sa = getattr(getattr(layers[0], "attention", None), "self", None)
        return all(hasattr(sa, n) for n in ("query", "key", "value", "num_attention_heads", "attention_head_size")) \
            and not getattr(getattr(base_model, "config", None), "is_decoder", False)

    def _positions(self, lengths: np.ndarray, cu: np.ndarray) -> np.ndarray:
        """Hugging Face's position ids of the real tokens of right-padded rows: 0..L-1 (BERT's absolute
        positions), or padding_idx + 1 + (0..L-1) for RoBERTa / XLM-R (create_position_ids_from_input_ids,
        whose cumulative count of non-pad tokens is exactly that on a right-padded row)."""
        n = int(cu[-1])
        pos = np.arange(n, dtype=np.int64) - np.repeat(cu[:-1], lengths)
        if hasattr(self.emb, "create_position_ids_from_input_ids"):
            pos += int(self.emb.padding_idx) + 1
        return pos

    def pack(self, input_ids, attention_mask, token_type_ids=None, device=None, granule: int = 0):
        """Host-side packing of right-padded tokenizer batches (host tensors / arrays (B, T), or lists of
        them -- several batches become one packed batch): the real tokens' ids, token types and
        positions plus the cumulative lengths, uploaded with ONE pinned asynchronous copy.  Returns the
        Packed batch forward_packed() takes.  granule > 0 (graph replay, GraphedForward): one more sequence of
        1..granule pad tokens (id 0) makes the token count a multiple of granule; its rows are computed and
        ignored (every sequence attends only to itself), and `lengths` keeps the real sequences only."""
        torch = self.torch
        many = isinstance(input_ids, (list, tuple))
        parts = zip(input_ids, attention_mask, token_type_ids if token_type_ids is not None else [None] * len(input_ids)) \
            if many else [(input_ids, attention_mask, token_type_ids)]
        ids_l, types_l, lens_l = [], [], []
        for ids, mask, types in parts:
            ids = np.asarray(ids)
            keep = np.asarray(mask).astype(bool, copy=False)
            lengths = keep.sum(1).astype(np.int64)
            if len(lengths) and not (keep == (np.arange(ids.shape[1])[None, :] < lengths[:, None])).all():
                raise ValueError("pack() needs right-padded rows (mask = a prefix of ones)")
            ids_l.append(ids[keep])
            types_l.append(np.asarray(types)[keep] if types is not None else None)
            lens_l.append(lengths)
        lengths = np.concatenate(lens_l) if lens_l else np.zeros(0, np.int64)
        real = lengths
        if granule > 0:
            n_real = int(lengths.sum())
            pad = granule - n_real % granule  # 1..granule: the pad sequence is never empty
            ids_l.append(np.zeros(pad, np.int64))
            types_l.append(None)
            lengths = np.concatenate([lengths, [pad]]).astype(np.int64)
        B = len(lengths)
        cu = np.zeros(B + 1, np.int64)
        cu[1:] = np.cumsum(lengths)
        n = int(cu[-1])
        buf = np.empty(3 * n + B + 1, np.int64)  # [ids | types | positions | cu]
        buf[:n] = np.concatenate(ids_l) if ids_l else 0
        o = n
        for t, ids in zip(types_l, ids_l):
            buf[o:o + len(ids)] = t if t is not None else 0
            o += len(ids)
        buf[2 * n:3 * n] = self._positions(lengths, cu)
        buf[3 * n:] = cu
        dev = torch.device(device) if device is not None else self.device
        t = torch.from_numpy(buf)
        if dev.type == "cuda":
            t = t.pin_memory()
        t = t.to(dev, non_blocking=dev.type == "cuda")
        return Packed(t[:n], t[n:2 * n], t[2 * n:3 * n], t[3 * n:].to(torch.int32), cu, real,
                      int(lengths.max()) if B else 0)

    def forward_packed(self, pk: "Packed"):
        """Last hidden state of the packed real tokens, (N, H) (row cu[b] + t is token t of sequence b)."""
        n = int(pk.cu_host[-1])
        for f in self.observers:  # (the pad sequence of a graph-shaped pack: executed, not real)
            f(len(pk.lengths), pk.max_len, pk.lengths, n - int(pk.lengths.sum()))
        x = self.emb(input_ids=pk.ids[None], token_type_ids=pk.types[None], position_ids=pk.pos[None])[0]
        return self._layers(x, pk.cu, pk.cu_host, pk.max_len, n)

    def _varlen_layer(self, scale: float, d: int) -> bool:
        """This layer's attention goes to the flash varlen kernel (its own 1/sqrt(d) scale), which reads the
        sequence offsets from the device tensor; else SDPA per sequence, sliced by the HOST offsets."""
        return self.varlen is not None and abs(scale * d ** 0.5 - 1.0) < 1e-6

    def graph_safe(self) -> bool:
        """Every layer takes the varlen branch, so a captured forward depends on the batch's offsets only through
        device tensors (GraphedForward copies them in before a replay).  The per-sequence SDPA fallback slices by
        host offsets, which a capture would bake in (a later batch of the same shape but other lengths
        then replayed the captured segmentation)."""
        return all(self._varlen_layer(scale, d) for _, _, _, d, scale, *_ in self.layers)

    def _layers(self, h, cu_t, cu_host, max_len, n):
        torch = self.torch
        from .. import _native

        n_seq = int(cu_t.shape[0]) - 1
        for w, b, nH, d, scale, attn_out, inter, out in self.layers:
            qkv2 = torch.nn.functional.linear(h, w, b)
            a = None
            if self.short_attn and max_len <= 64 and self._varlen_layer(scale, d):
                a = _native.attn_varlen(qkv2, cu_t, n_seq, nH, d, max_len, scale)  # None: not its shape
            if a is None:
                qkv = qkv2.view(n, 3, nH, d)
                q, k, v = qkv.unbind(1)  # strided views: the flash kernel takes them as they are (no copies)
                if self._varlen_layer(scale, d):
                    a = self.varlen(q, k, v, cu_t, cu_t, max_len, max_len)
                else:
                    a = _sdpa_per_sequence(q, k, v, cu_host, max_len, scale)
            h = attn_out(a.reshape(n, nH * d), h)
            h = out(inter(h), h)
        return h

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
        host = np.concatenate([idx_h, self._positions(lengths, cu), cu])
        t = torch.from_numpy(host)
        if dev.type == "cuda":
            t = t.pin_memory()
        t = t.to(dev, non_blocking=dev.type == "cuda")
        idx, pos, cu_t = t[:n], t[n:2 * n], t[2 * n:].to(torch.int32)
        ids_p = input_ids.reshape(-1).index_select(0, idx)
        types_p = token_type_ids.reshape(-1).index_select(0, idx) if token_type_ids is not None \
            else torch.zeros_like(ids_p)
        pk = Packed(ids_p, types_p, pos, cu_t, cu, lengths, int(lengths.max()) if B else 0)
        h = self.forward_packed(pk)
        seq = h.new_zeros(B * T, h.shape[-1])
        seq.index_copy_(0, idx, h)
        return seq.view(B, T, -1)


class GraphedForward:
    """forward_packed() replayed from HIP graphs: a query batch's forward is ~300 small kernels (24 layers at
    bge-large shape) whose host dispatch, not the GPU, bounds it (64 queries, ~900 tokens: 4.2 ms of host time
    for 4.0 ms of GPU time by events, 2.06 ms replayed; profiles/r04_embed_probe_bge-large_b64.json).  One graph
    per (sequences, tokens, max length) shape: batches are packed with a pad sequence up to a multiple of
    `granule` tokens (UnpaddedEncoder.pack) and the flash kernel's maximum length is rounded up to a power of two,
    so a stream of query batches falls into a few shapes.  Each graph is captured once (two warm-up forwards on a
    side stream first) into one shared memory pool; a call copies the packed ids / types / positions /
    offsets into the graph's static inputs on the current stream and replays it there.  The returned (N, H)
    hidden state is the graph's static output: valid until the next call on that stream.  Forwards above
    max_tokens run eagerly."""

    def __init__(self, enc: "UnpaddedEncoder", granule: int = 64, max_tokens: int = 8192, max_graphs: int = 64):
        self.enc = enc
        self.torch = enc.torch
        self.granule = int(granule)
        self.max_tokens = int(max_tokens)
        self.max_graphs = int(max_graphs)
        self.graphs: dict = {}
        self.pool = None
        self.replays = 0

    @staticmethod
    def _bucket_len(m: int) -> int:
        b = 32
        while b < m:
            b <<= 1
        return b

    def __call__(self, pk: "Packed"):
        n = int(pk.cu_host[-1])
        ml = self._bucket_len(pk.max_len)
        key = (len(pk.cu_host) - 1, n, ml)
        ent = self.graphs.get(key)
        if ent is None:
            if (n > self.max_tokens or not pk.ids.is_cuda or len(self.graphs) >= self.max_graphs
                    or not self.enc.graph_safe()):  # (host-sliced attention: never captured, see graph_safe)
                return self.enc.forward_packed(pk)
            ent = self.graphs[key] = self._capture(pk, ml)
        for f in self.enc.observers:  # (a replay runs no Python forward: report the shape here)
            f(len(pk.lengths), pk.max_len, pk.lengths, n - int(pk.lengths.sum()))
        ids, types, pos, cu, g, out = ent
        ids.copy_(pk.ids, non_blocking=True)
        types.copy_(pk.types, non_blocking=True)
        pos.copy_(pk.pos, non_blocking=True)
        cu.copy_(pk.cu, non_blocking=True)
        g.replay()
        self.replays += 1
        return out

    def _capture(self, pk: "Packed", ml: int):
        torch = self.torch
        dev = pk.ids.device
        ids, types, pos, cu = (x.clone() for x in (pk.ids, pk.types, pk.pos, pk.cu))
        spk = Packed(ids, types, pos, cu, pk.cu_host, pk.lengths, ml)
        side = torch.cuda.Stream(dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        obs, self.enc.observers = self.enc.observers, []  # (warm-up and capture are not forwards of a batch)
        try:
            with torch.cuda.stream(side):
                for _ in range(2):
                    self.enc.forward_packed(spk)
            torch.cuda.current_stream(dev).wait_stream(side)
            g = torch.cuda.CUDAGraph()
            # thread-local capture: the query coalescer captures on its worker thread while the event loop's thread
            # keeps making HIP calls for the store's searches; under the global mode those calls would
            # invalidate the capture or fail themselves
            with torch.cuda.graph(g, pool=self.pool, capture_error_mode="thread_local"):
                out = self.enc.forward_packed(spk)
        finally:
            self.enc.observers = obs
        if self.pool is None:
            self.pool = g.pool()
        return ids, types, pos, cu, g, out


class Packed(NamedTuple):
    """A packed batch on the device (ids, types, pos: (N,) int64; cu: (B+1,) int32) with its host
    offsets and lengths."""
    ids: Any
    types: Any
    pos: Any
    cu: Any
    cu_host: np.ndarray
    lengths: np.ndarray
    max_len: int


def first_tokens(h, cu_host, device=None):
    """(B, 1, H) view-like gather of each packed sequence's first token (the [CLS] / <s> position the
    poolers and classification heads read)."""
    import torch

    idx = torch.from_numpy(np.ascontiguousarray(cu_host[:-1]))
    if h.is_cuda:
        idx = idx.pin_memory().to(h.device, non_blocking=True)
    return h.index_select(0, idx)[:, None, :]


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

"""Algorithmic FLOPs of a BERT-shaped encoder forward (the C4 embedder, the C5 cross-encoder), counted
from the batches the model actually receives.

A forward pre-hook on the model records every batch's attention mask (kept on the device; the per-row
lengths are summed once at the end, so counting adds no host sync to the timed loop).  Per layer:
  * dense work (Q, K, V, O projections + the two FFN GEMMs): 2 * (4 H^2 + 2 H I) FLOP per token;
  * attention (Q K^T and P V): 2 * 2 * T_q * T_k * H per sequence (T_q = T_k = T).
``executed`` counts every position of the padded batch (what the GEMMs run on), ``useful`` only the real
tokens of each sequence (what an unpadded, length-exact forward would need).  Embedding lookups,
LayerNorms, GELU, the pooler / classifier head and the pooling kernel are not counted (O(H) per token
against O(H^2)): the figures are the MFMA-bound part of the forward, for MFMA roofline fractions
against the bf16 dense peak (2.5 PFLOP/s, MI355X_MICROARCH.md).
"""
from __future__ import annotations


class EncoderFlops:
    """Counts the forwards of `model`; pass `unpadded` (the embedder's / reranker's UnpaddedEncoder, which
    bypasses model.forward) to count those too -- there the executed FLOPs are the useful ones, plus the pad
    sequence a graph-replayed forward carries (encoder.GraphedForward)."""

    def __init__(self, model, unpadded=None):
        cfg = model.config
        self.L = int(cfg.num_hidden_layers)
        self.H = int(cfg.hidden_size)
        self.I = int(cfg.intermediate_size)
        self.masks = []
        self.unpadded = []  # host length arrays of unpadded forwards
        self.handle = model.register_forward_pre_hook(self._hook, with_kwargs=True)
        if unpadded is not None:
            unpadded.observers.append(lambda B, T, lengths, pad=0: self.unpadded.append((lengths.copy(), int(pad))))

    def _hook(self, module, args, kwargs):
        m = kwargs.get("attention_mask")
        if m is None and len(args) > 1:
            m = args[1]
        if m is not None:
            self.masks.append(m.detach().sum(dim=1))  # per-row real length (device tensor)
            self.masks.append(m.shape)

    def reset(self):
        self.masks = []
        self.unpadded = []

    def totals(self) -> dict:
        """{'executed': FLOP, 'useful': FLOP, 'tokens_padded', 'tokens_real', 'sequences'}."""
        import torch

        L, H, I = self.L, self.H, self.I
        dense = 2 * (4 * H * H + 2 * H * I)
        ex = us = tp = tr = ns = 0
        for lens, shape in zip(self.masks[0::2], self.masks[1::2]):
            B, T = int(shape[0]), int(shape[1])
            lens = lens.to(torch.float64).cpu()
            tp += B * T
            tr += int(lens.sum().item())
            ns += B
            ex += L * (B * T * dense + B * 4 * T * T * H)
            us += L * (float(lens.sum()) * dense + float((lens * lens).sum()) * 4 * H)
        for lens, pad in self.unpadded:  # real tokens (+ a graph replay's pad sequence: executed, not useful)
            n, sq = float(lens.sum()), float((lens.astype("float64") ** 2).sum())
            f = L * (n * dense + sq * 4 * H)
            ex += f + L * (pad * dense + pad * pad * 4 * H)
            us += f
            tp += int(n) + pad
            tr += int(n)
            ns += len(lens)
        return {"executed": float(ex), "useful": float(us), "tokens_padded": tp, "tokens_real": tr, "sequences": ns}

    def close(self):
        self.handle.remove()


def mfma_block(flops: dict, seconds: float, peak_tflops: float = 2500.0, what: str = "") -> dict:
    """The JSON object the benches print: achieved TFLOP/s over `seconds` and its fraction of the peak."""
    ex = flops["executed"] / seconds / 1e12 if seconds > 0 else 0.0
    us = flops["useful"] / seconds / 1e12 if seconds > 0 else 0.0
    return {"bound": "mfma", "achieved": round(ex, 1), "achieved_useful": round(us, 1), "peak": peak_tflops,
            "unit": "TFLOP/s", "frac": round(ex / peak_tflops, 4), "frac_useful": round(us / peak_tflops, 4),
            "flops_executed": flops["executed"], "flops_useful": flops["useful"],
            "tokens_padded": flops["tokens_padded"], "tokens_real": flops["tokens_real"],
            "sequences": flops["sequences"], "seconds": round(seconds, 4),
            "counted": what or "encoder GEMMs + attention products (tools/flops.py)"}

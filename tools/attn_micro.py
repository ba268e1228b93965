"""Micro-benchmark of the encoder attention variants at the C4 shape (bge-base: 12 heads x 64, a pack of
256 sequences of ~110-200 tokens, bf16): the masked SDPA Hugging Face's BERT runs today, SDPA with a
boolean mask, torch's varlen flash attention over the unpadded tokens, and unmasked SDPA (bound).
Prints one JSON line per variant: ms per call and TFLOP/s on the real (unpadded) tokens."""
import json
import time

import torch
import torch.nn.functional as F


def main():
    torch.manual_seed(0)
    dev = torch.device("cuda", 0)
    B, nH, d = 256, 12, 64
    lens = torch.randint(110, 200, (B,)).sort().values
    T = int(lens.max())
    q = torch.randn(B, nH, T, d, device=dev, dtype=torch.bfloat16)
    k, v = torch.randn_like(q), torch.randn_like(q)
    keep = torch.arange(T)[None, :] < lens[:, None]
    add_mask = torch.zeros(B, 1, 1, T, device=dev, dtype=torch.bfloat16)
    add_mask.masked_fill_(~keep.to(dev)[:, None, None, :], torch.finfo(torch.bfloat16).min)
    bool_mask = keep.to(dev)[:, None, None, :]
    real = float((lens.double() ** 2).sum()) * nH * 4 * d
    # unpadded (total, nH, d) + cumulative lengths
    qu = q.transpose(1, 2)[keep.to(dev)].contiguous()
    ku, vu = k.transpose(1, 2)[keep.to(dev)].contiguous(), v.transpose(1, 2)[keep.to(dev)].contiguous()
    cu = torch.zeros(B + 1, dtype=torch.int32)
    cu[1:] = lens.cumsum(0)
    cu = cu.to(dev)

    def timeit(fn, n=30):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(n):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t) / n * 1e3

    out = {}
    out["sdpa_additive_mask"] = timeit(lambda: F.scaled_dot_product_attention(q, k, v, attn_mask=add_mask))
    out["sdpa_bool_mask"] = timeit(lambda: F.scaled_dot_product_attention(q, k, v, attn_mask=bool_mask))
    out["sdpa_no_mask"] = timeit(lambda: F.scaled_dot_product_attention(q, k, v))
    try:
        from torch.nn.attention.varlen import varlen_attn

        out["varlen_unpadded"] = timeit(lambda: varlen_attn(qu, ku, vu, cu, cu, T, T))
        # the encoder's layout: q, k, v as strided views of one packed (N, 3, nH, d) QKV GEMM output
        qkv = torch.stack([qu, ku, vu], dim=1)
        qs, ks, vs = qkv[:, 0], qkv[:, 1], qkv[:, 2]
        try:
            out["varlen_unpadded_strided"] = timeit(lambda: varlen_attn(qs, ks, vs, cu, cu, T, T))
            out["varlen_strided_max_abs_diff"] = float((varlen_attn(qs, ks, vs, cu, cu, T, T).float()
                                                        - varlen_attn(qu, ku, vu, cu, cu, T, T).float()).abs().max())
        except Exception as e:  # noqa: BLE001
            out["varlen_strided_error"] = repr(e)[:300]
        out["varlen_unpadded_plus_copies"] = timeit(lambda: varlen_attn(qs.contiguous(), ks.contiguous(),
                                                                        vs.contiguous(), cu, cu, T, T))
        ref = F.scaled_dot_product_attention(q, k, v, attn_mask=add_mask).transpose(1, 2)[keep.to(dev)]
        got = varlen_attn(qu, ku, vu, cu, cu, T, T)
        out["varlen_max_abs_diff_vs_sdpa"] = float((got.float() - ref.float()).abs().max())
    except Exception as e:  # noqa: BLE001
        out["varlen_error"] = repr(e)[:300]
    for name, ms in list(out.items()):
        if name.endswith("mask") or name.startswith("varlen_unpadded"):
            print(json.dumps({"variant": name, "ms": round(ms, 3), "tflops_real": round(real / ms / 1e9, 1),
                              "B": B, "T": T, "heads": nH, "d": d}))
    print(json.dumps({k: v for k, v in out.items() if not isinstance(v, float) or "diff" in k}))


if __name__ == "__main__":
    main()

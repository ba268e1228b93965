"""GEMM ceiling at the encoder's shapes (bge-base: H = 768, I = 3072; bf16): y = x W^T + b for the
packed-token matrix x (M, K) at several M, through torch.nn.functional.linear (hipBLASLt) -- the
attainable MFMA rate the C4 / C5 forwards' GEMMs are measured against.  One JSON line per shape."""
import json
import sys
import time

import torch
import torch.nn.functional as F


def main():
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    Ms = [int(a) for a in sys.argv[1:]] or [8192, 32768, 131072, 524288]
    shapes = [("qkv", 768, 2304), ("attn_out", 768, 768), ("ffn_in", 768, 3072), ("ffn_out", 3072, 768)]
    for M in Ms:
        for name, K, N in shapes:
            x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
            w = torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02
            b = torch.randn(N, device=dev, dtype=torch.bfloat16)
            for _ in range(3):
                F.linear(x, w, b)
            torch.cuda.synchronize()
            n = max(5, int(2e13 / (2 * M * K * N)))
            t = time.perf_counter()
            for _ in range(n):
                F.linear(x, w, b)
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t) / n * 1e3
            tf = 2 * M * K * N / ms / 1e9
            print(json.dumps({"M": M, "gemm": name, "K": K, "N": N, "ms": round(ms, 4), "tflops": round(tf, 1),
                              "frac_of_2500": round(tf / 2500, 3)}), flush=True)
            del x, w, b


if __name__ == "__main__":
    main()

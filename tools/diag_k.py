"""Diagnostics: exact search time and guard failures across top-k on the bench corpus (synthetic,
counter-based), planted and isotropic query batches, synchronous path.
Usage: python tools/diag_k.py [rows] [dim] [dtype] [metric] [allowed_frac] [deleted_frac] [ks]
(allowed_frac < 1: a random row mask passed to every search; deleted_frac > 0: that many random rows
removed first; ks: comma-separated top-k values)"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "youtu-rag_amd"), REPO]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from hiprag import _native, synth  # noqa: E402

N = int(float(sys.argv[1])) if len(sys.argv) > 1 else 10_000_000
D = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
DT = sys.argv[3] if len(sys.argv) > 3 else "bf16"
MET = sys.argv[4] if len(sys.argv) > 4 else "cosine"
ALLOWED = float(sys.argv[5]) if len(sys.argv) > 5 else 1.0
DELETED = float(sys.argv[6]) if len(sys.argv) > 6 else 0.0
KS = [int(x) for x in sys.argv[7].split(",")] if len(sys.argv) > 7 else [10, 32, 45, 100, 128]
B = 64
dev = torch.device("cuda", 0)
st = torch.cuda.current_stream(dev).cuda_stream
idx = _native.NativeIndex(D, DT, MET)
idx.reserve(N)
idx.add_synthetic(0, 0, N)
torch.cuda.synchronize()
rng = np.random.default_rng(9)
if DELETED > 0:
    idx.remove(np.nonzero(rng.random(N) < DELETED)[0])
mask_ptr, mask_d = 0, None
if ALLOWED < 1.0:
    bits = np.packbits(rng.random(N) < ALLOWED, bitorder="little")
    bits = np.concatenate([bits, np.zeros((-len(bits)) % 8, np.uint8)])
    mask_d = torch.from_numpy(bits.view(np.int64).copy()).to(dev)
    mask_ptr = mask_d.data_ptr()
planted = torch.from_numpy(synth.planted_queries(0, N, D, B, qseed=77)[0]).to(dev)
iso = torch.randn((B, D), generator=torch.Generator().manual_seed(3)).to(dev)
for name, q in (("planted", planted), ("isotropic", iso)):
    for k in KS:
        s = torch.empty((B, k), dtype=torch.float32, device=dev)
        r = torch.empty((B, k), dtype=torch.int64, device=dev)
        idx.search_device(q.data_ptr(), B, k, s.data_ptr(), r.data_ptr(), mask_ptr=mask_ptr, stream=st)  # warm (graph capture etc.)
        torch.cuda.synchronize()
        before = idx.stats()
        t0 = time.perf_counter()
        for _ in range(3):
            idx.search_device(q.data_ptr(), B, k, s.data_ptr(), r.data_ptr(), mask_ptr=mask_ptr, stream=st)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) * 1e3 / 3
        after = idx.stats()
        tot, mx = idx.last_candidates()
        print(f"{DT} {MET} allowed {ALLOWED:g} deleted {DELETED:g} {name:9s} k={k:3d} kc={_native.kc_for_k(k, D):3d}: {ms:7.2f} ms/batch, guard failures "
              f"{(after['guard_failures'] - before['guard_failures']) / 3:.1f}/{B}, exhaustive "
              f"{(after['exhaustive'] - before['exhaustive']) / 3:.1f}, candidates/query {tot / B:.0f} max {mx}",
              flush=True)

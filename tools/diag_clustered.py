"""Diagnostics: exact search on a clustered corpus -- guard failures, fallback cost."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "youtu-rag_amd"), REPO]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from hiprag import _native  # noqa: E402

N, D, B = int(float(sys.argv[1])), 1024, 64
C, spread = int(sys.argv[2]), float(sys.argv[3])
dtype = sys.argv[4] if len(sys.argv) > 4 else "f16"
dev = torch.device("cuda", 0)
st = torch.cuda.current_stream(dev).cuda_stream
centers = torch.empty((C, D), dtype=torch.float32, device=dev)
_native.gen_rows_device(7, 0, C, D, centers.data_ptr(), st)
centers = torch.nn.functional.normalize(centers, dim=1)


def rows(i0, i1):
    noise = torch.empty((i1 - i0, D), dtype=torch.float32, device=dev)
    _native.gen_rows_device(11, i0, i1 - i0, D, noise.data_ptr(), st)
    c = (torch.arange(i0, i1, device=dev, dtype=torch.int64) * 2654435761) % C
    return centers[c] + spread * torch.nn.functional.normalize(noise, dim=1)


flat = _native.NativeIndex(D, dtype, "cosine")
flat.reserve(N)
for i in range(0, N, 1 << 18):
    x = rows(i, min(N, i + (1 << 18))).contiguous()
    flat.add_device(x.data_ptr(), x.shape[0], st)
g = torch.Generator(device=dev)
g.manual_seed(5)
j = torch.randint(0, N, (B,), generator=g, device=dev)
q = (torch.cat([rows(int(r), int(r) + 1) for r in j.tolist()]) + 0.1 * torch.randn((B, D), generator=g, device=dev)).contiguous()
if os.environ.get("DIAG_QUERIES") == "mixed":  # bench_ivf's batches: half planted, half isotropic
    q = torch.cat([q[: B // 2], torch.randn((B - B // 2, D), generator=g, device=dev)]).contiguous()
for k in (10, 100):
    kc = _native.kc_for_k(k)
    cand = torch.empty((B, kc, 2), dtype=torch.float64, device=dev)
    bound = torch.empty(B, dtype=torch.float64, device=dev)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    flat.search_shard(q.data_ptr(), B, k, kc, 0, cand.data_ptr(), bound.data_ptr(), stream=st)
    torch.cuda.synchronize()
    t_main = time.perf_counter() - t0
    s = torch.empty((B, k), dtype=torch.float32, device=dev)
    r = torch.empty((B, k), dtype=torch.int64, device=dev)
    kth = torch.empty(B, dtype=torch.float64, device=dev)
    fail = torch.empty(B, dtype=torch.int32, device=dev)
    _native.merge_candidates(0, cand.data_ptr(), bound.data_ptr(), 1, B, kc, k, s.data_ptr(), r.data_ptr(),
                             kth.data_ptr(), fail.data_ptr(), stream=st)
    torch.cuda.synchronize()
    nf = int(fail.sum())
    gap = (kth - bound).cpu().numpy()
    tot, mx = flat.last_candidates()
    t0 = time.perf_counter()
    flat.search_device(q.data_ptr(), B, k, s.data_ptr(), r.data_ptr(), stream=st)
    torch.cuda.synchronize()
    t_full = time.perf_counter() - t0
    print(f"k={k} kc={kc}: main pass {t_main * 1e3:.2f} ms, full search {t_full * 1e3:.2f} ms, guard failures {nf}/{B}, "
          f"kth-bound gap median {np.median(gap):.2e} min {gap.min():.2e}, candidates/query {tot / B:.0f} max {mx}",
          flush=True)
    print(f"  index stats after k={k}: {flat.stats()}", flush=True)

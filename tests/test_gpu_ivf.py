"""GPU parity of the IVF-flat candidate generation (hiprag.ivf, hr_ivf.hip; BASELINE config 5):
given the index's trained centroids and list assignment, the probed lists and the returned ids /
scores are identical to the oracle's IVF restatement (oracle/ref_numpy.ivf_search); with
nprobe = nlist the IVF search IS the exact search (identical to NativeIndex.search)."""
import numpy as np
import pytest

import oracle  # noqa: F401
from oracle import ref_numpy as R

pytestmark = pytest.mark.gpu


def _clustered(rng, n, dim, n_centers=40, spread=0.35):
    centers = rng.standard_normal((n_centers, dim)).astype(np.float32)
    centers /= np.linalg.norm(centers, axis=1, keepdims=True)
    lab = rng.integers(0, n_centers, n)
    x = centers[lab] + spread * rng.standard_normal((n, dim)).astype(np.float32) / np.sqrt(dim)
    return x.astype(np.float32)


def _build(x, nlist, dtype, metric="cosine", chunk=1 << 18):
    import torch

    from hiprag.ivf import IvfIndex

    xd = torch.from_numpy(x).cuda()
    ivf = IvfIndex(x.shape[1], nlist, dtype=dtype, metric=metric)
    ivf.train(xd[:: max(1, len(x) // (nlist * 40))], iters=8, seed=1)
    ivf.build(len(x), lambda i, j: xd[i:j], chunk=chunk)
    return ivf


@pytest.mark.parametrize("dim,dtype,n,nlist,B,k", [(128, "bf16", 20000, 64, 32, 10), (96, "f16", 9000, 50, 17, 100),
                                                   (256, "f32", 6000, 24, 40, 32), (1024, "f16", 30000, 128, 64, 100),
                                                   (384, "bf16", 5000, 32, 20, 10), (768, "f16", 8000, 40, 33, 50),
                                                   (1100, "bf16", 3000, 16, 9, 10)])
def test_ivf_matches_oracle(dim, dtype, n, nlist, B, k):
    import torch

    rng = np.random.default_rng(dim + nlist)
    x = _clustered(rng, n, dim)
    ivf = _build(x, nlist, dtype, chunk=7000)  # several build chunks
    j = rng.choice(n, B // 2, replace=False)
    q = np.concatenate([x[j] + 0.02 * rng.standard_normal((len(j), dim)).astype(np.float32),
                        rng.standard_normal((B - len(j), dim)).astype(np.float32)]).astype(np.float32)
    stored = R.process_rows(x, "cosine", dtype)
    cent = ivf.centroids[:, :dim].cpu().numpy()
    row_list = ivf.lists_of_rows.cpu().numpy()
    for nprobe in (1, 5, nlist):
        qd = torch.from_numpy(q).cuda()
        cand = torch.empty((B, k, 2), dtype=torch.float64, device="cuda")
        bound = torch.empty(B, dtype=torch.float64, device="cuda")
        probes = torch.empty((B, nprobe, 2), dtype=torch.float64, device="cuda")
        ivf.search_candidates(qd, k, nprobe, cand, bound, probes=probes)
        torch.cuda.synchronize()
        s_ref, r_ref, p_ref = R.ivf_search(stored, dtype, R.process_queries(q, "cosine"), cent, row_list, nprobe, k)
        np.testing.assert_array_equal(probes.view(torch.int64)[..., 1].cpu().numpy(), p_ref)
        np.testing.assert_array_equal(cand.view(torch.int64)[..., 1].cpu().numpy(), r_ref)
        np.testing.assert_array_equal(cand[..., 0].cpu().numpy(), s_ref)
        assert torch.all(torch.isneginf(bound))
    # all lists probed: the IVF search is the exact search
    s, r = ivf.search(torch.from_numpy(q).cuda(), k, nlist)
    from hiprag import _native

    flat = _native.NativeIndex(dim, dtype, "cosine")
    flat.add(x)
    s_f, r_f = flat.search(q, k)
    np.testing.assert_array_equal(r.cpu().numpy(), r_f)
    np.testing.assert_array_equal(s.cpu().numpy(), s_f)


def test_ivf_ties_padding_dot_and_synthetic():
    """Duplicate rows tie-break by id, k beyond the visible rows pads with -1, dot metric, and the
    device synthetic build equals a host build of the same rows."""
    import torch

    from hiprag.ivf import IvfIndex

    rng = np.random.default_rng(7)
    dim, n, nlist = 64, 3000, 16
    x = _clustered(rng, n, dim, n_centers=8)
    dup = rng.choice(n, 50, replace=False)
    x[dup] = x[dup[0]]
    ivf = _build(x, nlist, "bf16", metric="ip")
    q = x[dup[:1]].copy()
    s_ref, r_ref, _ = R.ivf_search(R.process_rows(x, "ip", "bf16"), "bf16", q, ivf.centroids[:, :dim].cpu().numpy(),
                                   ivf.lists_of_rows.cpu().numpy(), 2, 700)
    s, r = ivf.search(torch.from_numpy(q).cuda(), 700, 2)
    np.testing.assert_array_equal(r.cpu().numpy(), r_ref)
    np.testing.assert_array_equal(s.cpu().numpy().astype(np.float64), s_ref.astype(np.float32).astype(np.float64))
    assert (r_ref[0] == -1).any()  # fewer visible rows than k
    # synthetic device build == host build of the same generator rows
    a = IvfIndex(dim, 8, dtype="f16")
    raw = R.gen_rows(3, 100, 4000, dim)
    a.train(torch.from_numpy(raw).cuda(), iters=4, seed=0)
    a.build_synthetic(3, 100, 4000)
    b = IvfIndex(dim, 8, dtype="f16")
    b.centroids = a.centroids.clone()
    rd = torch.from_numpy(raw).cuda()
    b.build(4000, lambda i, j: rd[i:j], id_offset=100)
    assert torch.equal(a.ids, b.ids) and torch.equal(a.list_tiles, b.list_tiles)
    qq = torch.from_numpy(raw[:8] + 0.1).cuda()
    sa, ra = a.search(qq, 10, 3)
    sb, rb = b.search(qq, 10, 3)
    assert torch.equal(ra, rb) and torch.equal(sa, sb)
    assert int(ra.min()) >= 100

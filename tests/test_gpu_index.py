"""GPU parity tests: libhiprag.so (through its C ABI) against the CPU oracle and the
golden vectors produced by the reference's own VectorRetriever (tests/golden/).

Bar: returned rows identical (bit-exact, including the (score desc, row asc) tie
order); scores identical to the oracle's fp64 canonical scores cast to fp32, and
within 1e-5 of the golden fp64 scores (north_star tolerance).
"""
import hashlib
import json
import os

import numpy as np
import pytest

import oracle
from oracle import ref_numpy as R

pytestmark = pytest.mark.gpu

SCORE_TOL = 1e-5


@pytest.fixture(scope="module")
def native():
    from hiprag import _native

    _native.load_library()
    assert _native.device_count() >= 1, "no HIP device visible"
    return _native


def _stored_as_f32(stored, dtype):
    return R.dequantize(stored, dtype)


def _planted_queries(corpus_rows_f32, B, rng, noise=0.05):
    n, dim = corpus_rows_f32.shape
    idx = rng.choice(n, B, replace=False)
    base = corpus_rows_f32[idx] / np.linalg.norm(corpus_rows_f32[idx], axis=1, keepdims=True)
    eps = rng.standard_normal((B, dim)).astype(np.float32)
    eps /= np.linalg.norm(eps, axis=1, keepdims=True)
    return (base + noise * eps).astype(np.float32)


def _check(s_gpu, r_gpu, s_ref, r_ref):
    np.testing.assert_array_equal(r_gpu, r_ref)
    valid = r_ref >= 0
    np.testing.assert_array_equal(s_gpu[valid], s_ref[valid].astype(np.float32))
    assert np.all(np.isneginf(s_gpu[~valid]))


# ---------------------------------------------------------------- K1+K2 storage
@pytest.mark.parametrize("dim,dtype,metric", [(128, "bf16", "cosine"), (768, "bf16", "cosine"), (1024, "bf16", "cosine"),
                                              (1024, "f16", "cosine"), (1024, "f32", "cosine"), (100, "bf16", "cosine"),
                                              (128, "bf16", "ip")])
def test_store_bit_exact(native, dim, dtype, metric, golden_dir):
    n = 4096 if dim >= 768 else 1000
    idx = native.NativeIndex(dim, dtype, metric)
    idx.add_synthetic(0, 0, n)
    got = idx.get_rows(np.arange(n))
    ref = _stored_as_f32(oracle.c_build_synthetic(0, 0, n, dim, dtype, metric), dtype)
    np.testing.assert_array_equal(got.view(np.uint32), ref.view(np.uint32))
    sha = json.load(open(os.path.join(golden_dir, "corpus_sha256.json")))
    key = f"seed0_rows{n}_dim{dim}_{dtype}_{metric}"
    if key in sha:
        st = R.quantize(got, dtype)
        assert hashlib.sha256(st.tobytes()).hexdigest() == sha[key]
    # explicit fp32 rows go through the same K1+K2 path
    idx2 = native.NativeIndex(dim, dtype, metric)
    idx2.add(R.gen_rows(0, 0, n, dim))
    np.testing.assert_array_equal(idx2.get_rows(np.arange(n)).view(np.uint32), ref.view(np.uint32))


# ---------------------------------------------------------------- golden vectors
def test_c1_golden(native, golden_dir):
    d = np.load(os.path.join(golden_dir, "c1_retrieval.npz"))
    meta = json.load(open(os.path.join(golden_dir, "c1_retrieval.json")))
    idx = native.NativeIndex(128, "f32", "cosine")
    idx.add(d["corpus"])
    s, r = idx.search(d["queries"], 5)
    for b, res in enumerate(meta["results"]["thr0"]):
        assert [f"chunk_{x}" for x in r[b]] == [e["chunk_id"] for e in res]
        np.testing.assert_allclose(s[b], [e["score"] for e in res], atol=SCORE_TOL, rtol=0)
    allowed = np.array([m["group"] == "g1" for m in meta["metas"]])
    s, r = idx.search(d["queries"], 5, oracle.mask_from_bool(allowed))
    for b, res in enumerate(meta["results"]["filtered_g1"]):
        assert [f"chunk_{x}" for x in r[b] if x >= 0] == [e["chunk_id"] for e in res]
        np.testing.assert_allclose(s[b][: len(res)], [e["score"] for e in res], atol=SCORE_TOL, rtol=0)


@pytest.mark.parametrize("dtype", ["f32", "bf16"])
def test_ties_golden(native, golden_dir, dtype):
    d = np.load(os.path.join(golden_dir, "ties.npz"))
    meta = json.load(open(os.path.join(golden_dir, "ties.json")))
    corpus = R.gen_rows(7, 0, 20000, 256)
    for s_, dst in zip(d["dup_src"], d["dup_dst"]):
        corpus[dst] = corpus[s_]
    idx = native.NativeIndex(256, dtype, "cosine")
    idx.add(corpus)
    s, r = idx.search(d["queries"], 10)
    stored = R.process_rows(corpus, "cosine", dtype)
    s_ref, r_ref = oracle.c_search(stored, dtype, R.process_queries(d["queries"], "cosine"), 10)
    _check(s, r, s_ref, r_ref)
    if dtype == "f32":  # the golden vectors were produced on the fp32 store
        for b, res in enumerate(meta["results"]):
            assert [f"chunk_{x}" for x in r[b]] == [e["chunk_id"] for e in res]
            np.testing.assert_allclose(s[b], [e["score"] for e in res], atol=SCORE_TOL, rtol=0)


# ---------------------------------------------------------------- random sweeps vs the oracle
CASES = [
    (64, "bf16", 2000, 1, 10), (128, "bf16", 5000, 16, 5), (384, "bf16", 20000, 33, 10), (768, "bf16", 30000, 64, 10),
    (1024, "bf16", 30000, 64, 32), (1024, "bf16", 7000, 100, 10), (768, "f16", 20000, 64, 10),
    (1024, "f32", 20000, 48, 10), (200, "f32", 3000, 7, 3), (2048, "bf16", 5000, 40, 10), (96, "f16", 777, 5, 32),
]


@pytest.mark.parametrize("dim,dtype,n,B,k", CASES)
def test_random_vs_oracle(native, dim, dtype, n, B, k):
    rng = np.random.default_rng(dim * 7 + B)
    idx = native.NativeIndex(dim, dtype, "cosine")
    idx.add_synthetic(3, 0, n)
    raw = R.gen_rows(3, 0, n, dim)
    q = np.concatenate([_planted_queries(raw, B // 2, rng), rng.standard_normal((B - B // 2, dim)).astype(np.float32)])
    s, r = idx.search(q, k)
    stored = oracle.c_build_synthetic(3, 0, n, dim, dtype, "cosine")
    s_ref, r_ref = oracle.c_search(stored, dtype, R.process_queries(q, "cosine"), k)
    _check(s, r, s_ref, r_ref)


# top-k beyond 32 (kb_file_search recall 15 x 3, rerank top-100): ceil(kc/32) row parts of group maxima
LARGE_K = [(768, "bf16", 40000, 64, 45), (1024, "bf16", 30000, 64, 100), (256, "f16", 9000, 33, 128),
           (384, "f32", 20000, 20, 64), (128, "bf16", 3000, 5, 128), (64, "bf16", 150, 3, 100),
           (2304, "bf16", 20000, 64, 100), (2048, "f16", 12000, 96, 32)]


@pytest.mark.parametrize("dim,dtype,n,B,k", LARGE_K)
def test_large_k_vs_oracle(native, dim, dtype, n, B, k):
    rng = np.random.default_rng(dim + k)
    idx = native.NativeIndex(dim, dtype, "cosine")
    idx.add_synthetic(6, 0, n)
    raw = R.gen_rows(6, 0, n, dim)
    q = np.concatenate([_planted_queries(raw, B // 2, rng), rng.standard_normal((B - B // 2, dim)).astype(np.float32)])
    allowed = rng.random(n) < 0.7
    stored = oracle.c_build_synthetic(6, 0, n, dim, dtype, "cosine")
    for mask in (None, allowed):
        s, r = idx.search(q, k, None if mask is None else oracle.mask_from_bool(mask))
        s_ref, r_ref = oracle.c_search(stored, dtype, R.process_queries(q, "cosine"), k,
                                       None if mask is None else oracle.mask_from_bool(mask))
        _check(s, r, s_ref, r_ref)


def test_dynamic_tail_and_pipelined_workspaces_vs_oracle(native):
    """A shard large enough for the FILTER scan's dynamic tail (>= 8 tiles per wave; the pool has
    an odd tile count, so the last run is one tile), searched synchronously and through the
    pipelined two-workspace path (scan stream + tail stream) with several batches in flight,
    with and without a row mask: every batch identical to the oracle."""
    torch = pytest.importorskip("torch")
    from hiprag.dist import ShardedSearch

    dim, n, B, k = 64, 600_032, 64, 10
    idx = native.NativeIndex(dim, "bf16", "cosine")
    idx.add_synthetic(21, 0, n)
    raw = R.gen_rows(21, 0, n, dim)
    rng = np.random.default_rng(5)
    qs = [np.concatenate([_planted_queries(raw, B // 2, rng), rng.standard_normal((B - B // 2, dim)).astype(np.float32)])
          for _ in range(4)]
    stored = oracle.c_build_synthetic(21, 0, n, dim, "bf16", "cosine")
    refs = [oracle.c_search(stored, "bf16", R.process_queries(q, "cosine"), k) for q in qs]
    for q, (s_ref, r_ref) in zip(qs, refs):
        s, r = idx.search(q, k)
        _check(s, r, s_ref, r_ref)
    ss = ShardedSearch(idx, 0, max_batch=B, device=torch.device("cuda", 0))
    assert ss.tail is not None
    s_out = torch.empty((len(qs), B, k), dtype=torch.float32, device="cuda")
    r_out = torch.empty((len(qs), B, k), dtype=torch.int64, device="cuda")
    for i, q in enumerate(qs):  # submit finalizes the slot it reuses
        ss.submit(torch.from_numpy(q).cuda(), k, s_out=s_out[i], r_out=r_out[i])
    ss.finalize_all()
    torch.cuda.synchronize()
    for i, (s_ref, r_ref) in enumerate(refs):
        _check(s_out[i].cpu().numpy(), r_out[i].cpu().numpy(), s_ref, r_ref)
    allowed = rng.random(n) < 0.5
    mask = oracle.mask_from_bool(allowed)
    s, r = idx.search(qs[0], k, mask)
    _check(s, r, *oracle.c_search(stored, "bf16", R.process_queries(qs[0], "cosine"), k, mask))


@pytest.mark.parametrize("metric", ["cosine", "l2"])
def test_early_sample_pipelined_vs_oracle(native, metric):
    """Queries ready by event on a shard large enough (>= 8 sample sizes) for the early SAMPLE:
    query prep + SAMPLE run on the index's pre stream beside the previous batch's FILTER, and each
    workspace's FILTER on its own stream.  Batches of different shapes (B = 64 / 20 -> 2 / 1 query
    blocks, k = 10 / 100 -> 1 / 5 row parts, with and without a device row mask) alternate over the
    two workspaces: all identical to the oracle (cosine and euclidean)."""
    torch = pytest.importorskip("torch")
    from hiprag.dist import ShardedSearch

    dim, n = 64, 1_100_000
    idx = native.NativeIndex(dim, "bf16", metric)
    idx.add_synthetic(23, 0, n)
    raw = R.gen_rows(23, 0, n, dim)
    stored = oracle.c_build_synthetic(23, 0, n, dim, "bf16", metric)
    rng = np.random.default_rng(8)
    dense = rng.random(n) < 0.6
    docs = np.zeros(n, bool)  # a few documents' chunks: the device mask builds a tile list
    for lo in (1000, 500_000, 1_050_000):
        docs[lo:lo + 3000] = True
    masks_h = {"dense": oracle.mask_from_bool(dense), "docs": oracle.mask_from_bool(docs)}
    masks_d = {kk: torch.from_numpy(v.view(np.int64)).cuda() for kk, v in masks_h.items()}
    plan = [(64, 10, None), (64, 10, "dense"), (20, 10, None), (64, 100, "docs"), (64, 10, "docs"), (20, 100, "dense"),
            (64, 10, None), (64, 10, "docs"), (64, 10, None)]
    qs = [np.concatenate([_planted_queries(raw, B // 2, rng), rng.standard_normal((B - B // 2, dim)).astype(np.float32)])
          for B, _, _ in plan]
    q_dev = [torch.from_numpy(q).cuda() for q in qs]
    outs = [(torch.empty((B, k), dtype=torch.float32, device="cuda"), torch.empty((B, k), dtype=torch.int64, device="cuda"))
            for B, k, _ in plan]
    q_ready = torch.cuda.Event()
    q_ready.record()
    ss = ShardedSearch(idx, 0, max_batch=64, max_k=100, device=torch.device("cuda", 0))
    for (B, k, mk), q, (s_o, r_o) in zip(plan, q_dev, outs):
        ss.submit(q, k, s_out=s_o, r_out=r_o, mask_ptr=masks_d[mk].data_ptr() if mk else 0, q_ready=q_ready)
    ss.finalize_all()
    torch.cuda.synchronize()
    for (B, k, mk), q, (s_o, r_o) in zip(plan, qs, outs):
        s_ref, r_ref = oracle.c_search(stored, "bf16", R.process_queries(q, metric), k, masks_h[mk] if mk else None,
                                       metric=metric)
        _check(s_o.cpu().numpy(), r_o.cpu().numpy(), s_ref, r_ref)
    # the synchronous device entry point with the sparse device mask (tile list on the scan stream)
    s_d = torch.empty((64, 10), dtype=torch.float32, device="cuda")
    r_d = torch.empty((64, 10), dtype=torch.int64, device="cuda")
    idx.search_device(q_dev[0].data_ptr(), 64, 10, s_d.data_ptr(), r_d.data_ptr(), mask_ptr=masks_d["docs"].data_ptr(),
                      stream=torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    s_ref, r_ref = oracle.c_search(stored, "bf16", R.process_queries(qs[0], metric), 10, masks_h["docs"], metric=metric)
    _check(s_d.cpu().numpy(), r_d.cpu().numpy(), s_ref, r_ref)


@pytest.mark.parametrize("metric", ["cosine", "l2"])
def test_early_sample_clusters_dups_tombstones_vs_oracle(native, metric):
    """The early-SAMPLE pipelined path on a shard with tight clusters spread over it (20k rows
    around each of three rows, so the sampled tiles and the FILTER's row groups are full of near
    ties), 200 exact duplicates and 5000 tombstones, with planted / cluster / duplicate / isotropic
    query batches over both workspaces, twice: every batch identical to the oracle, the queries the
    guard cannot settle answered by the exact fallback."""
    torch = pytest.importorskip("torch")
    from hiprag.dist import ShardedSearch

    dim, n, B, k = 64, 1_100_000, 64, 10
    rng = np.random.default_rng(31)
    raw = R.gen_rows(29, 0, n, dim)
    centers = []
    for j in rng.choice(n, 3, replace=False):  # clusters of 20k rows around three rows
        c = raw[j] / np.linalg.norm(raw[j])
        pos = rng.choice(n, 20_000, replace=False)
        noise = rng.standard_normal((len(pos), dim)).astype(np.float32)
        raw[pos] = c + 0.02 * noise / np.linalg.norm(noise, axis=1, keepdims=True)
        centers.append(c)
    dup = rng.choice(n, 200, replace=False)
    raw[dup] = raw[dup[0]]
    idx = native.NativeIndex(dim, "bf16", metric)
    idx.add(raw)
    gone = rng.choice(n, 5000, replace=False)
    idx.remove(gone)
    live = np.ones(n, bool)
    live[gone] = False
    stored = R.process_rows(raw, metric, "bf16")
    cl = np.stack([centers[i % 3] + 0.01 * rng.standard_normal(dim).astype(np.float32) for i in range(B)])
    qs = [np.concatenate([_planted_queries(raw, B // 2, rng), rng.standard_normal((B - B // 2, dim)).astype(np.float32)]),
          cl.astype(np.float32), np.concatenate([raw[dup[:8]], rng.standard_normal((B - 8, dim)).astype(np.float32)]),
          rng.standard_normal((B, dim)).astype(np.float32)]
    q_dev = [torch.from_numpy(np.ascontiguousarray(q)).cuda() for q in qs]
    outs = [(torch.empty((B, k), dtype=torch.float32, device="cuda"), torch.empty((B, k), dtype=torch.int64, device="cuda"))
            for _ in qs]
    ready = torch.cuda.Event()
    ready.record()
    ss = ShardedSearch(idx, 0, max_batch=B, device=torch.device("cuda", 0))
    for rep in range(2):  # both workspaces, twice
        for q, (s_o, r_o) in zip(q_dev, outs):
            ss.submit(q, k, s_out=s_o, r_out=r_o, q_ready=ready)
        ss.finalize_all()
        torch.cuda.synchronize()
        for q, (s_o, r_o) in zip(qs, outs):
            s_ref, r_ref = oracle.c_search(stored, "bf16", R.process_queries(q, metric), k, oracle.mask_from_bool(live),
                                           metric=metric)
            _check(s_o.cpu().numpy(), r_o.cpu().numpy(), s_ref, r_ref)


def test_periodic_clusters_spread_over_waves(native):
    """Rows whose cluster repeats with a period of 4096 rows (128 tiles, a factor of the scan's wave
    count): the FILTER's round-robin dealing rotates each round's positions, so a cluster's rows (a
    query's candidates) reach every wave instead of the few waves whose tiles share its residue -- their
    32-slot private regions stayed below capacity and the guard held for k = 10 (and the row parts of
    k = 100 keep contiguous ranges).  Results identical to the oracle either way."""
    dim, n, B, C = 64, 6_250_000, 64, 4096
    rng = np.random.default_rng(17)
    centers = rng.standard_normal((C, dim)).astype(np.float32)
    centers /= np.linalg.norm(centers, axis=1, keepdims=True)
    noise = R.gen_rows(41, 0, n, dim)
    noise /= np.linalg.norm(noise, axis=1, keepdims=True)
    raw = centers[(np.arange(n, dtype=np.int64) * 2654435761) % C] + 0.7 * noise
    idx = native.NativeIndex(dim, "bf16", "cosine")
    idx.add(raw)
    stored = R.process_rows(raw, "cosine", "bf16")
    q = (raw[rng.choice(n, B, replace=False)] + 0.1 * rng.standard_normal((B, dim))).astype(np.float32)
    for k in (10, 100):
        before = idx.stats()["guard_failures"]
        s, r = idx.search(q, k)
        _check(s, r, *oracle.c_search(stored, "bf16", R.process_queries(q, "cosine"), k))
        failed = idx.stats()["guard_failures"] - before
        assert failed <= B // 8, (k, failed)


@pytest.mark.parametrize("dtype,metric,k", [("bf16", "cosine", 10), ("bf16", "cosine", 100), ("f32", "cosine", 32),
                                            ("f16", "cosine", 45), ("bf16", "ip", 45), ("bf16", "l2", 10)])
def test_selective_filter_tile_list_vs_oracle(native, dtype, metric, k):
    """Row masks that leave at most half the tiles (a few documents' contiguous chunks; 1 % of the
    rows at random; a handful of rows; nothing): the scans visit only the listed tiles.  Identical
    to the oracle, including k > 32 (row parts over the listed tiles) and deleted rows."""
    dim, n, B = 128, 200_000, 24
    idx = native.NativeIndex(dim, dtype, metric)
    idx.add_synthetic(17, 0, n)
    idx.remove(np.arange(5000, 5100))  # deleted rows inside an allowed range
    rng = np.random.default_rng(k)
    raw = R.gen_rows(17, 0, n, dim)
    q = np.concatenate([_planted_queries(raw, B // 2, rng), rng.standard_normal((B - B // 2, dim)).astype(np.float32)])
    stored = oracle.c_build_synthetic(17, 0, n, dim, dtype, metric)
    live = np.ones(n, bool)
    live[5000:5100] = False
    docs = np.zeros(n, bool)
    for lo in (4900, 77_777, 150_001):
        docs[lo:lo + 700] = True
    few = np.zeros(n, bool)
    few[rng.choice(n, 7, replace=False)] = True
    for allowed in (docs, rng.random(n) < 0.01, few, np.zeros(n, bool)):
        mask = oracle.mask_from_bool(allowed)
        s, r = idx.search(q, k, mask)
        s_ref, r_ref = oracle.c_search(stored, dtype, R.process_queries(q, metric), k,
                                       oracle.mask_from_bool(allowed & live), metric=metric)
        _check(s, r, s_ref, r_ref)


@pytest.mark.parametrize("dtype,metric", [("bf16", "cosine"), ("f32", "cosine"), ("f16", "cosine"), ("bf16", "euclidean"), ("bf16", "ip")])
def test_topk_beyond_max_k_exhaustive(native, dtype, metric):
    """top_k > HR_MAX_K (Chroma has no n_results cap): the exhaustive exact path, identical to the
    oracle, with and without a mask, including k beyond the number of allowed rows (-inf / -1).
    (The synthetic rows are raw-scale: euclidean keeps them unnormalised, so not in f16.)"""
    dim, n, B = 96, 3000, 5
    m = "l2" if metric == "euclidean" else metric
    idx = native.NativeIndex(dim, dtype, metric)
    idx.add_synthetic(12, 0, n)
    rng = np.random.default_rng(3)
    raw = R.gen_rows(12, 0, n, dim)
    q = np.concatenate([_planted_queries(raw, 3, rng), rng.standard_normal((B - 3, dim)).astype(np.float32)])
    stored = oracle.c_build_synthetic(12, 0, n, dim, dtype, m)
    qp = R.process_queries(q, m)
    allowed = rng.random(n) < 0.1  # ~300 allowed rows: k = 500 runs past them
    for k, mask in ((129, None), (500, None), (500, oracle.mask_from_bool(allowed))):
        s, r = idx.search(q, k, mask)
        s_ref, r_ref = oracle.c_search(stored, dtype, qp, k, mask, metric=m)
        _check(s, r, s_ref, r_ref)
    assert (r[:, -1] == -1).all()


def test_large_k_massive_ties(native):
    """300 identical rows, k = 100: the 100 lowest duplicate rows, via the exact fallback."""
    dim, n = 128, 8000
    raw = R.gen_rows(12, 0, n, dim)
    dups = np.sort(np.random.default_rng(4).choice(n, 300, replace=False))
    raw[dups] = raw[dups[0]]
    idx = native.NativeIndex(dim, "bf16", "cosine")
    idx.add(raw)
    s, r = idx.search(raw[dups[:1]].copy(), 100)
    np.testing.assert_array_equal(r[0], dups[:100])


@pytest.mark.parametrize("dtype,k", [("bf16", 10), ("f32", 128), ("f16", 45)])
def test_exhaustive_exact_when_window_overflows(native, dtype, k):
    """Concentrated embeddings (every row within the error bound of the k-th score, as a
    random-init transformer produces) and 2000 exact duplicates: the collect window overflows
    its buffer and the exhaustive exact pass answers -- still identical to the oracle."""
    dim, n = 256, 12000
    rng = np.random.default_rng(21)
    base = rng.standard_normal(dim).astype(np.float32)
    raw = (base + 1e-4 * rng.standard_normal((n, dim))).astype(np.float32)
    dups = np.sort(rng.choice(n, 2000, replace=False))
    raw[dups] = raw[dups[0]]
    idx = native.NativeIndex(dim, dtype, "cosine")
    idx.add(raw)
    gone = rng.choice(n, 500, replace=False)
    idx.remove(gone)
    allowed = rng.random(n) < 0.8
    eff = allowed.copy()
    eff[gone] = False
    q = np.stack([raw[dups[0]], base + 1e-4 * rng.standard_normal(dim).astype(np.float32), rng.standard_normal(dim)])
    q = q.astype(np.float32)
    stored = R.process_rows(raw, "cosine", dtype)
    for m in (None, allowed):
        s, r = idx.search(q, k, None if m is None else oracle.mask_from_bool(m))
        s_ref, r_ref = oracle.c_search(stored, dtype, R.process_queries(q, "cosine"), k,
                                       oracle.mask_from_bool(eff if m is not None else ~np.isin(np.arange(n), gone)))
        _check(s, r, s_ref, r_ref)


def test_ip_metric(native):
    rng = np.random.default_rng(5)
    x = rng.standard_normal((3000, 128)).astype(np.float32) * rng.uniform(0.1, 3.0, (3000, 1)).astype(np.float32)
    q = rng.standard_normal((9, 128)).astype(np.float32)
    idx = native.NativeIndex(128, "bf16", "ip")
    idx.add(x)
    s, r = idx.search(q, 10)
    s_ref, r_ref = oracle.c_search(R.process_rows(x, "ip", "bf16"), "bf16", q, 10)
    _check(s, r, s_ref, r_ref)


def test_mask_remove_and_incremental_add(native):
    rng = np.random.default_rng(11)
    dim, n = 256, 9000
    raw = R.gen_rows(5, 0, n, dim)
    idx = native.NativeIndex(dim, "bf16", "cosine")
    idx.add(raw[:4000])
    idx.add(raw[4000:7001])
    idx.add(raw[7001:])
    gone = rng.choice(n, 700, replace=False)
    idx.remove(gone)
    assert idx.size() == (n, n - 700)
    allowed = rng.random(n) < 0.4
    q = _planted_queries(raw, 20, rng)
    s, r = idx.search(q, 10, oracle.mask_from_bool(allowed))
    eff = allowed.copy()
    eff[gone] = False
    stored = R.process_rows(raw, "cosine", "bf16")
    s_ref, r_ref = oracle.c_search(stored, "bf16", R.process_queries(q, "cosine"), 10, oracle.mask_from_bool(eff))
    _check(s, r, s_ref, r_ref)


def test_empty_small_and_ragged(native):
    idx = native.NativeIndex(64, "bf16", "cosine")
    q = np.ones((2, 64), np.float32)
    s, r = idx.search(q, 5)
    assert (r == -1).all() and np.isneginf(s).all()
    raw = R.gen_rows(1, 0, 3, 64)
    idx.add(raw)
    s, r = idx.search(q, 5)
    s_ref, r_ref = oracle.c_search(R.process_rows(raw, "cosine", "bf16"), "bf16", R.process_queries(q, "cosine"), 5)
    _check(s, r, s_ref, r_ref)
    assert (r[:, 3:] == -1).all()
    idx.remove([0, 1, 2])
    s, r = idx.search(q, 5)
    assert (r == -1).all()
    s, r = idx.search(q, native.HR_MAX_K + 1)  # no top-k cap (the exhaustive path beyond HR_MAX_K)
    assert (r == -1).all() and np.isneginf(s).all()
    with pytest.raises(ValueError):
        idx.search(q, 0)
    with pytest.raises(ValueError):
        idx.search(np.ones((1, 63), np.float32), 5)


def test_massive_ties_use_exact_fallback(native):
    """100 identical rows (> kc = 32 candidates): the guard fails and the collect pass
    must return the 10 lowest duplicate rows."""
    dim, n = 128, 5000
    raw = R.gen_rows(9, 0, n, dim)
    dups = np.sort(np.random.default_rng(2).choice(n, 100, replace=False))
    raw[dups] = raw[dups[0]]
    idx = native.NativeIndex(dim, "bf16", "cosine")
    idx.add(raw)
    q = raw[dups[:1]].copy()
    s, r = idx.search(q, 10)
    s_ref, r_ref = oracle.c_search(R.process_rows(raw, "cosine", "bf16"), "bf16", R.process_queries(q, "cosine"), 10)
    _check(s, r, s_ref, r_ref)
    np.testing.assert_array_equal(r[0], dups[:10])


def test_graph_replay_vs_oracle(native):
    """hr_index_search from the second call of a (B, k) shape on replays a captured HIP graph
    (hr_index_graph_replays): its results must be the oracle's on every call -- new queries each
    time, after an add (rows grow: the graph is recaptured), after a remove (live bits change on
    the device: the same graph still applies), with a guard failure (massive ties: the fallback
    runs after the replay), and beside masked and large-k calls that take the normal path."""
    rng = np.random.default_rng(21)
    dim, n = 256, 6000
    raw = R.gen_rows(13, 0, n + 1500, dim)
    dups = np.sort(rng.choice(n, 60, replace=False))
    raw[dups] = raw[dups[0]]
    idx = native.NativeIndex(dim, "bf16", "cosine")
    idx.add(raw[:n])
    alive = np.zeros(n + 1500, bool)
    alive[:n] = True
    stored = R.process_rows(raw, "cosine", "bf16")

    def run(q, k, mask=None):
        s, r = idx.search(q, k, None if mask is None else oracle.mask_from_bool(mask))
        eff = alive[: idx.size()[0]] if mask is None else (alive[: idx.size()[0]] & mask)
        s_ref, r_ref = oracle.c_search(stored[: idx.size()[0]], "bf16", R.process_queries(q, "cosine"), k,
                                       oracle.mask_from_bool(eff))
        _check(s, r, s_ref, r_ref)
        return r

    r0 = idx.graph_replays()
    for it in range(4):
        run(_planted_queries(raw[:n], 16, rng), 10)
        run(_planted_queries(raw[:n], 1, rng), 5)
    assert idx.graph_replays() - r0 >= 6  # each shape: first call normal, then replays
    # ties: the replayed pass flags the guard, the exact fallback finishes the query
    q_t = np.concatenate([raw[dups[:1]], _planted_queries(raw[:n], 15, rng)])
    before = idx.stats()["guard_failures"]
    for _ in range(2):
        r = run(q_t, 10)
        np.testing.assert_array_equal(r[0], dups[:10])
    assert idx.stats()["guard_failures"] >= before + 2
    # a masked call and a k > HR_MAX_K call in between take the normal path
    run(_planted_queries(raw[:n], 16, rng), 10, rng.random(n) < 0.5)
    run(_planted_queries(raw[:n], 2, rng), native.HR_MAX_K + 3)
    # remove: live bits change in place, the captured graph reads them at run time
    gone = rng.choice(n, 500, replace=False)
    idx.remove(gone)
    alive[gone] = False
    run(_planted_queries(raw[:n], 16, rng), 10)
    # add: the row count changes, the graph is recaptured for the new size
    idx.add(raw[n:])
    alive[n:] = True
    for _ in range(3):
        run(_planted_queries(raw, 16, rng), 10)
    assert idx.graph_replays() - r0 >= 10


def test_save_load_roundtrip(native, tmp_path):
    raw = R.gen_rows(4, 0, 1500, 192)
    idx = native.NativeIndex(192, "f16", "cosine")
    idx.add(raw)
    idx.remove([3, 77])
    p = str(tmp_path / "x.hri")
    idx.save(p)
    idx2 = native.NativeIndex.load(p, dim=192, dtype="f16", metric="cosine")
    assert idx2.size() == (1500, 1498)
    q = raw[:4] + 0.01
    np.testing.assert_array_equal(idx.search(q, 8)[1], idx2.search(q, 8)[1])


# ---------------------------------------------------------------- device + shard paths
def test_device_and_sharded_merge(native):
    torch = pytest.importorskip("torch")
    dim, n, B, k, kc = 512, 12000, 24, 10, 32
    raw = R.gen_rows(8, 0, n, dim)
    full = native.NativeIndex(dim, "bf16", "cosine")
    full.add(raw)
    rng = np.random.default_rng(3)
    q = _planted_queries(raw, B, rng)
    s_host, r_host = full.search(q, k)
    qd = torch.from_numpy(q).cuda()
    sd = torch.empty((B, k), dtype=torch.float32, device="cuda")
    rd = torch.empty((B, k), dtype=torch.int64, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    full.search_device(qd.data_ptr(), B, k, sd.data_ptr(), rd.data_ptr(), stream=st)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(rd.cpu().numpy(), r_host)
    np.testing.assert_array_equal(sd.cpu().numpy(), s_host)
    # two row shards + device merge == one index
    cut = 5003
    shards = [native.NativeIndex(dim, "bf16", "cosine") for _ in range(2)]
    shards[0].add(raw[:cut])
    shards[1].add(raw[cut:])
    cand = torch.empty((2, B, kc, 2), dtype=torch.float64, device="cuda")
    bounds = torch.empty((2, B), dtype=torch.float64, device="cuda")
    for g, (sh, off) in enumerate(zip(shards, [0, cut])):
        sh.search_shard(qd.data_ptr(), B, k, kc, off, cand[g].data_ptr(), bounds[g].data_ptr(), stream=st)
    torch.cuda.synchronize()
    kth = torch.empty(B, dtype=torch.float64, device="cuda")
    fail = torch.empty(B, dtype=torch.int32, device="cuda")
    native.merge_candidates(0, cand.data_ptr(), bounds.data_ptr(), 2, B, kc, k, sd.data_ptr(), rd.data_ptr(),
                            kth.data_ptr(), fail.data_ptr(), stream=st)
    torch.cuda.synchronize()
    assert fail.sum().item() == 0
    np.testing.assert_array_equal(rd.cpu().numpy(), r_host)
    np.testing.assert_array_equal(sd.cpu().numpy(), s_host)


def test_sharded_merge_large_k(native):
    torch = pytest.importorskip("torch")
    dim, n, B, k = 256, 20000, 40, 100
    kc = native.kc_for_k(k)
    raw = R.gen_rows(13, 0, n, dim)
    q = _planted_queries(raw, B, np.random.default_rng(8))
    s_ref, r_ref = oracle.c_search(R.process_rows(raw, "cosine", "bf16"), "bf16", R.process_queries(q, "cosine"), k)
    cuts = [0, 6001, 13007, n]
    qd = torch.from_numpy(q).cuda()
    st = torch.cuda.current_stream().cuda_stream
    G = len(cuts) - 1
    cand = torch.empty((G, B, kc, 2), dtype=torch.float64, device="cuda")
    bounds = torch.empty((G, B), dtype=torch.float64, device="cuda")
    shards = []
    for g in range(G):
        sh = native.NativeIndex(dim, "bf16", "cosine")
        sh.add(raw[cuts[g]:cuts[g + 1]])
        sh.search_shard(qd.data_ptr(), B, k, kc, cuts[g], cand[g].data_ptr(), bounds[g].data_ptr(), stream=st)
        shards.append(sh)
    sd = torch.empty((B, k), dtype=torch.float32, device="cuda")
    rd = torch.empty((B, k), dtype=torch.int64, device="cuda")
    kth = torch.empty(B, dtype=torch.float64, device="cuda")
    fail = torch.empty(B, dtype=torch.int32, device="cuda")
    native.merge_candidates(0, cand.data_ptr(), bounds.data_ptr(), G, B, kc, k, sd.data_ptr(), rd.data_ptr(),
                            kth.data_ptr(), fail.data_ptr(), stream=st)
    torch.cuda.synchronize()
    ok = fail.cpu().numpy() == 0
    assert ok.mean() > 0.9  # planted queries: the guard should almost always hold
    np.testing.assert_array_equal(rd.cpu().numpy()[ok], r_ref[ok])
    np.testing.assert_array_equal(sd.cpu().numpy()[ok], s_ref[ok].astype(np.float32))


@pytest.mark.parametrize("dim", [256, 1024])
def test_shard_search_f32_kc256_query_groups(native, dim):
    """fp32 rows, 128 queries, kc = HR_MAX_KC = 256 (8 row parts: more than the 128-query FILTER's 7, so the
    FILTER is k_scan<F32, QB = 2> with two query groups), through hr_index_search_shard + the merge: ids and
    scores identical to the oracle wherever the guard holds, and the rest through the collect path of the
    synchronous search."""
    torch = pytest.importorskip("torch")
    n, B, k, kc = 30_011, 128, 128, 256
    raw = R.gen_rows(17, 0, n, dim)
    q = np.concatenate([_planted_queries(raw, B // 2, np.random.default_rng(dim)),
                        np.random.default_rng(dim + 1).standard_normal((B // 2, dim)).astype(np.float32)])
    stored = R.process_rows(raw, "cosine", "f32")
    s_ref, r_ref = oracle.c_search(stored, "f32", R.process_queries(q, "cosine"), k)
    idx = native.NativeIndex(dim, "f32", "cosine")
    idx.add(raw)
    qd = torch.from_numpy(q).cuda()
    st = torch.cuda.current_stream().cuda_stream
    cand = torch.empty((1, B, kc, 2), dtype=torch.float64, device="cuda")
    bounds = torch.empty((1, B), dtype=torch.float64, device="cuda")
    w0 = idx.wide_launches()
    idx.search_shard(qd.data_ptr(), B, k, kc, 0, cand[0].data_ptr(), bounds[0].data_ptr(), stream=st)
    sd = torch.empty((B, k), dtype=torch.float32, device="cuda")
    rd = torch.empty((B, k), dtype=torch.int64, device="cuda")
    kth = torch.empty(B, dtype=torch.float64, device="cuda")
    fail = torch.empty(B, dtype=torch.int32, device="cuda")
    native.merge_candidates(0, cand.data_ptr(), bounds.data_ptr(), 1, B, kc, k, sd.data_ptr(), rd.data_ptr(),
                            kth.data_ptr(), fail.data_ptr(), stream=st)
    torch.cuda.synchronize()
    assert idx.wide_launches() == w0  # 8 parts: the query groups, not the 128-query FILTER
    ok = fail.cpu().numpy() == 0
    assert ok.mean() > 0.5
    np.testing.assert_array_equal(rd.cpu().numpy()[ok], r_ref[ok])
    np.testing.assert_array_equal(sd.cpu().numpy()[ok], s_ref[ok].astype(np.float32))
    s, r = idx.search(q, k)
    _check(s, r, s_ref, r_ref)
    idx.close()


def test_pool_normalize_matches_torch(native):
    torch = pytest.importorskip("torch")
    B, T, H, n_instr = 5, 37, 768, 6
    g = torch.Generator().manual_seed(0)
    hidden = torch.randn(B, T, H, generator=g).to(torch.bfloat16)
    mask = torch.ones(B, T, dtype=torch.int32)
    mask[1, 20:] = 0
    mask[3, 9:] = 0
    ref_mask = mask.clone()
    ref_mask[:, :n_instr] = 0
    s = torch.sum(hidden.float() * ref_mask.unsqueeze(-1).float(), dim=1)
    d = ref_mask.sum(dim=1, keepdim=True).float()
    ref = torch.nn.functional.normalize(s / d, dim=-1)
    hd, md = hidden.cuda(), mask.cuda()
    out = torch.empty(B, H, device="cuda")
    native.pool_normalize(hd.data_ptr(), "bf16", md.data_ptr(), B, T, H, n_instr, out.data_ptr(),
                          stream=torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    torch.testing.assert_close(out.cpu(), ref, atol=1e-5, rtol=1e-5)


# ---------------------------------------------------------------- guard rigor
@pytest.mark.parametrize("dim,dtype,B", [(128, "bf16", 16), (200, "f32", 7), (1024, "f32", 48), (1024, "bf16", 64),
                                         (768, "f16", 40)])
def test_approx_error_within_guard_bound(native, dim, dtype, B):
    """Every row's approximate MFMA score lies within E_q of its exact canonical score --
    the premise of the exactness guard (DESIGN.md "Exactness guard")."""
    n = 3000
    rng = np.random.default_rng(dim + B)
    idx = native.NativeIndex(dim, dtype, "cosine")
    idx.add_synthetic(3, 0, n)
    raw = R.gen_rows(3, 0, n, dim)
    q = np.concatenate([_planted_queries(raw, B // 2, rng), rng.standard_normal((B - B // 2, dim)).astype(np.float32)])
    approx, E = idx.debug_approx(q)
    stored = oracle.c_build_synthetic(3, 0, n, dim, dtype, "cosine")
    exact = R.exact_scores(stored, dtype, R.process_queries(q, "cosine"))
    err = np.abs(approx.astype(np.float64) - exact).max(axis=1)
    print(f"{dim}/{dtype}: max |approx-exact| = {err.max():.3e}, min E = {E.min():.3e}")
    assert np.all(err <= E), (err, E)


# ---------------------------------------------------------------- euclidean (Chroma hnsw "l2")
# similarity = 1 - squared L2 distance (chroma_store.py:48-53, :135) over raw vectors; the oracle's
# exact restatement (hr_oracle.c row_score) is the reference for ids and bits.  chromadb is not
# importable here, so the L2 convention is pinned by the reference's own mapping, not a fixture.
def _embedding_like(rng, n, dim, scale=1.0):
    x = rng.standard_normal((n, dim)).astype(np.float32)
    x /= np.linalg.norm(x, axis=1, keepdims=True)
    return (x * (scale * (0.5 + rng.random((n, 1))))).astype(np.float32)  # norms spread over [0.5, 1.5]·scale


L2_CASES = [(128, "bf16", 5000, 16, 10), (768, "f16", 20000, 64, 10), (1024, "f32", 8000, 33, 5),
            (256, "bf16", 9000, 20, 100), (96, "bf16", 700, 5, 32), (1024, "bf16", 600_000 // 20, 64, 10),
            # more than 64 queries: the 128-query FILTER with euclidean scores (2 q.x - |x|^2)
            (1024, "bf16", 40_001, 128, 10), (768, "f32", 20_000, 200, 16), (512, "f16", 9_000, 97, 20)]


@pytest.mark.parametrize("dim,dtype,n,B,k", L2_CASES)
def test_euclidean_vs_oracle(native, dim, dtype, n, B, k):
    rng = np.random.default_rng(dim * 3 + k)
    x = _embedding_like(rng, n, dim, scale=3.0)
    idx = native.NativeIndex(dim, dtype, "l2")
    idx.add(x)
    j = rng.choice(n, B // 2, replace=False)
    q = np.concatenate([x[j] + 0.05 * rng.standard_normal((len(j), dim)).astype(np.float32),
                        _embedding_like(rng, B - B // 2, dim, scale=3.0)]).astype(np.float32)
    stored = R.process_rows(x, "l2", dtype)
    allowed = rng.random(n) < 0.6
    for mask in (None, oracle.mask_from_bool(allowed)):
        s, r = idx.search(q, k, mask)
        s_ref, r_ref = oracle.c_search(stored, dtype, q, k, mask, metric="l2")
        _check(s, r, s_ref, r_ref)
    np.testing.assert_array_equal(r[: len(j), 0][allowed[j]], j[allowed[j]])  # a planted row is its query's nearest


@pytest.mark.parametrize("dim,dtype", [(128, "bf16"), (768, "f16"), (200, "f32")])
def test_euclidean_approx_error_within_guard_bound(native, dim, dtype):
    """Scan score 2 q̂.x - |x|^2 (fp32) within E of the exact 2 q.x - |x|^2 for every row."""
    rng = np.random.default_rng(dim)
    n, B = 3000, 24
    x = _embedding_like(rng, n, dim, scale=2.0)
    idx = native.NativeIndex(dim, dtype, "l2")
    idx.add(x)
    q = _embedding_like(rng, B, dim, scale=2.0)
    approx, E = idx.debug_approx(q)
    xs = R.dequantize(R.process_rows(x, "l2", dtype), dtype).astype(np.float64)
    qd = q.astype(np.float64)
    exact = 2.0 * R.canon_sum(qd[:, None, :] * xs[None]) - R.canon_sum(xs * xs)[None, :]
    err = np.abs(approx.astype(np.float64) - exact).max(axis=1)
    print(f"l2 {dim}/{dtype}: max |approx-exact| = {err.max():.3e}, min E = {E.min():.3e}")
    assert np.all(err <= E), (err, E)


def test_euclidean_ties_save_load_and_shards(native, tmp_path):
    """300 identical rows (exhaustive exact pass for k = 100), a save/load round trip (row norms
    rebuilt on load) and a two-shard device merge, all equal to the oracle."""
    torch = pytest.importorskip("torch")
    dim, n = 128, 8000
    rng = np.random.default_rng(11)
    x = _embedding_like(rng, n, dim)
    dups = np.sort(rng.choice(n, 300, replace=False))
    x[dups] = x[dups[0]]
    idx = native.NativeIndex(dim, "bf16", "l2")
    idx.add(x)
    stored = R.process_rows(x, "l2", "bf16")
    s, r = idx.search(x[dups[:1]].copy(), 100)
    s_ref, r_ref = oracle.c_search(stored, "bf16", x[dups[:1]], 100, metric="l2")
    _check(s, r, s_ref, r_ref)
    np.testing.assert_array_equal(r[0], dups[:100])
    p = str(tmp_path / "l2.hri")
    idx.save(p)
    idx2 = native.NativeIndex.load(p, dim=dim, dtype="bf16", metric="l2")
    q = _embedding_like(rng, 24, dim)
    s1, r1 = idx.search(q, 10)
    s2, r2 = idx2.search(q, 10)
    np.testing.assert_array_equal(r1, r2)
    np.testing.assert_array_equal(s1, s2)
    _check(s1, r1, *oracle.c_search(stored, "bf16", q, 10, metric="l2"))
    cut, kc, B, k = 3001, 32, 24, 10
    shards = [native.NativeIndex(dim, "bf16", "l2") for _ in range(2)]
    shards[0].add(x[:cut])
    shards[1].add(x[cut:])
    qd = torch.from_numpy(q).cuda()
    cand = torch.empty((2, B, kc, 2), dtype=torch.float64, device="cuda")
    bounds = torch.empty((2, B), dtype=torch.float64, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    for g, (sh, off) in enumerate(zip(shards, [0, cut])):
        sh.search_shard(qd.data_ptr(), B, k, kc, off, cand[g].data_ptr(), bounds[g].data_ptr(), stream=st)
    sd = torch.empty((B, k), dtype=torch.float32, device="cuda")
    rd = torch.empty((B, k), dtype=torch.int64, device="cuda")
    kth = torch.empty(B, dtype=torch.float64, device="cuda")
    fail = torch.empty(B, dtype=torch.int32, device="cuda")
    native.merge_candidates(0, cand.data_ptr(), bounds.data_ptr(), 2, B, kc, k, sd.data_ptr(), rd.data_ptr(),
                            kth.data_ptr(), fail.data_ptr(), stream=st)
    torch.cuda.synchronize()
    assert fail.sum().item() == 0
    np.testing.assert_array_equal(rd.cpu().numpy(), r1)
    np.testing.assert_array_equal(sd.cpu().numpy(), s1)


# ---------------------------------------------------------------- seeded fuzz over the parameter space
def _fuzz_cases(n_cases=36, seed=2024):
    rng = np.random.default_rng(seed)
    dims = [1, 17, 63, 64, 65, 130, 255, 384, 1000, 1024, 2560]
    out = []
    for i in range(n_cases):
        dim = int(rng.choice(dims))
        dtype = str(rng.choice(["f32", "bf16", "f16"]))
        metric = str(rng.choice(["cosine", "ip", "l2"]))
        if dtype == "f32" and dim > 1280:
            dim = 1000  # fp32 query tiles of 2560-d do not fit the LDS-resident plan
        B = int(rng.choice([1, 7, 33, 64, 65, 100]))
        k = int(rng.choice([1, 5, 10, 32, 33, 64, 100, 128]))
        n = int(rng.integers(1, 12000))
        out.append((i, dim, dtype, metric, B, k, n, bool(rng.random() < 0.4)))
    return out


@pytest.mark.parametrize("case", _fuzz_cases(), ids=lambda c: "-".join(map(str, c)))
def test_fuzz_vs_oracle(native, case):
    """Random (dim, dtype, metric, B, k, n, mask) combinations, including B > 64 (query chunks),
    n < k, odd dims and every metric: ids and bits equal to the oracle."""
    i, dim, dtype, metric, B, k, n, use_mask = case
    rng = np.random.default_rng(i)
    x = rng.standard_normal((n, dim)).astype(np.float32)
    if metric != "cosine":
        x *= (0.5 + rng.random((n, 1))).astype(np.float32)
    idx = native.NativeIndex(dim, dtype, metric)
    try:
        idx.add(x)
    except ValueError:  # plan limits (dim x dtype) are reported, not silently degraded
        pytest.skip("unsupported plan")
    j = rng.integers(0, n, B)
    q = (x[j] + 0.1 * rng.standard_normal((B, dim))).astype(np.float32)
    mask = oracle.mask_from_bool(rng.random(n) < 0.5) if use_mask else None
    try:
        s, r = idx.search(q, k, mask)
    except ValueError:
        pytest.skip("unsupported plan")
    stored = R.process_rows(x, metric, dtype)
    s_ref, r_ref = oracle.c_search(stored, dtype, R.process_queries(q, metric), k, mask, metric=metric)
    _check(s, r, s_ref, r_ref)


def _fuzz_filter_cases(n_cases=20, seed=77):
    rng = np.random.default_rng(seed)
    out = []
    for i in range(n_cases):
        dim = int(rng.choice([17, 64, 130, 384, 1024]))
        dtype = str(rng.choice(["f32", "bf16", "f16"]))
        metric = str(rng.choice(["cosine", "ip", "l2"]))
        B = int(rng.choice([1, 9, 64, 70]))
        k = int(rng.choice([1, 10, 33, 100, 128, 129, 300]))
        n = int(rng.integers(2000, 40000))
        kind = str(rng.choice(["sparse", "docs", "half", "none"]))
        out.append((i, dim, dtype, metric, B, k, n, kind))
    return out


@pytest.mark.parametrize("case", _fuzz_filter_cases(), ids=lambda c: "-".join(map(str, c)))
def test_fuzz_filters_and_large_k_vs_oracle(native, case):
    """Random combinations over the filter paths -- sparse random masks and document ranges
    (tile lists), dense masks (full scan) -- and k across the scan / exhaustive boundary
    (k > HR_MAX_K), with deleted rows: ids and bits equal to the oracle."""
    i, dim, dtype, metric, B, k, n, kind = case
    rng = np.random.default_rng(1000 + i)
    x = rng.standard_normal((n, dim)).astype(np.float32)
    if metric != "cosine":
        x *= (0.5 + rng.random((n, 1))).astype(np.float32)
    idx = native.NativeIndex(dim, dtype, metric)
    idx.add(x)
    dead = rng.choice(n, n // 50, replace=False)
    idx.remove(dead)
    live = np.ones(n, bool)
    live[dead] = False
    allowed = np.ones(n, bool)
    if kind == "sparse":
        allowed = rng.random(n) < 0.005
    elif kind == "docs":
        allowed = np.zeros(n, bool)
        for lo in rng.integers(0, n, 3):
            allowed[lo:lo + int(rng.integers(1, 400))] = True
    elif kind == "half":
        allowed = rng.random(n) < 0.5
    mask = None if kind == "none" else oracle.mask_from_bool(allowed)
    j = rng.integers(0, n, B)
    q = (x[j] + 0.1 * rng.standard_normal((B, dim))).astype(np.float32)
    s, r = idx.search(q, k, mask)
    stored = R.process_rows(x, metric, dtype)
    s_ref, r_ref = oracle.c_search(stored, dtype, R.process_queries(q, metric), k,
                                   oracle.mask_from_bool(allowed & live), metric=metric)
    _check(s, r, s_ref, r_ref)


# ---------------------------------------------------------------- query groups: > 64 queries per corpus pass
@pytest.mark.parametrize("dim,dtype,n,B,k", [(1024, "bf16", 60_000, 256, 10), (768, "f16", 40_000, 200, 100),
                                             (256, "bf16", 30_000, 65, 32), (1024, "bf16", 9_000, 128, 128),
                                             (128, "f32", 20_000, 150, 10), (1024, "bf16", 100_000, 128, 10),
                                             (768, "bf16", 50_000, 100, 20), (1024, "f16", 30_000, 150, 5),
                                             (768, "f16", 20_000, 192, 32), (768, "f32", 20_000, 130, 45)])
def test_query_groups_vs_oracle(native, dim, dtype, n, B, k):
    """B > 64: ceil(B/64) workgroup groups stream the same tiles in one pass (one XCD per range
    block), each with 64 queries in LDS; per-group private candidate regions, thresholds and
    dynamic-tail counters.  Identical to the oracle, with and without a mask, and to the same
    queries searched 64 at a time."""
    rng = np.random.default_rng(dim + B + k)
    idx = native.NativeIndex(dim, dtype, "cosine")
    idx.add_synthetic(8, 0, n)
    raw = R.gen_rows(8, 0, n, dim)
    q = np.concatenate([_planted_queries(raw, B // 2, rng), rng.standard_normal((B - B // 2, dim)).astype(np.float32)])
    stored = oracle.c_build_synthetic(8, 0, n, dim, dtype, "cosine")
    qn = R.process_queries(q, "cosine")
    allowed = rng.random(n) < 0.6
    for m in (None, allowed):
        mk = None if m is None else oracle.mask_from_bool(m)
        s, r = idx.search(q, k, mk)
        _check(s, r, *oracle.c_search(stored, dtype, qn, k, mk))
        parts = [idx.search(q[i:i + 64], k, mk) for i in range(0, B, 64)]
        np.testing.assert_array_equal(r, np.concatenate([p[1] for p in parts]))


@pytest.mark.parametrize("dim,dtype,metric", [(1024, "bf16", "cosine"), (768, "f16", "cosine"), (1024, "bf16", "ip"),
                                              # fp32 rows form query groups where the 128-query FILTER could take
                                              # them; a tile list (selective mask) or k = 1 then falls back to
                                              # k_scan<F32, QB = 2> with ng > 1
                                              (256, "f32", "cosine"), (768, "f32", "cosine"), (1024, "f32", "ip")])
def test_query_group_edges_vs_oracle(native, dim, dtype, metric):
    """Query groups (65..256 queries per corpus pass, k <= 32, D = 768 / 1024): fewer tiles than
    workgroups, ragged ranges, a selective filter (tile list), a removed stretch, and massive ties that
    overflow the private candidate regions (the guard then sends the query to the exact fallback) --
    identical to the oracle every time."""
    rng = np.random.default_rng(dim + 3)
    for n, B, k in ((500, 65, 10), (9_001, 128, 32), (70_000, 256, 1), (40_000, 130, 16)):
        raw = R.gen_rows(31, 0, n, dim)
        if n == 40_000:  # 600 copies of one row inside one workgroup's range
            raw[1000:1600] = raw[1000]
        idx = native.NativeIndex(dim, dtype, metric)
        idx.add(raw)
        stored = R.process_rows(raw, metric, dtype)
        q = np.concatenate([_planted_queries(raw, B // 2, rng), rng.standard_normal((B - B // 2, dim)).astype(np.float32)])
        if n == 40_000:
            q[:3] = raw[1000]
        qn = R.process_queries(q, metric)
        sel = np.zeros(n, bool)
        sel[n // 3: n // 3 + max(40, n // 50)] = True
        for mask in (None, sel):
            mk = None if mask is None else oracle.mask_from_bool(mask)
            s, r = idx.search(q, k, mk)
            _check(s, r, *oracle.c_search(stored, dtype, qn, k, mk, metric=metric))
        if n == 40_000:
            s, r = idx.search(q, k)
            np.testing.assert_array_equal(r[0], np.arange(1000, 1000 + k))
        gone = np.arange(n // 2, n // 2 + n // 10)
        idx.remove(gone)
        live = np.ones(n, bool)
        live[gone] = False
        s, r = idx.search(q, k)
        _check(s, r, *oracle.c_search(stored, dtype, qn, k, oracle.mask_from_bool(live), metric=metric))


# ---------------------------------------------------------------- the 128-query FILTER (hr_wide.hip)
@pytest.mark.parametrize("dim,dtype,n,B,k", [(256, "bf16", 20_011, 128, 10), (512, "f16", 33_333, 97, 16),
                                             (768, "bf16", 41_000, 129, 20), (1024, "bf16", 70_001, 256, 10),
                                             (1024, "f16", 3_000, 80, 5), (512, "bf16", 64, 128, 3),
                                             (1024, "bf16", 1_000_003, 128, 10), (1024, "f32", 50_001, 128, 10),
                                             (768, "f32", 20_000, 200, 16), (256, "f32", 3_001, 65, 5),
                                             # row parts (kc > 32: 2..7 parts of 32 groups; 16-bit rows up to 3
                                             # parts and 128 queries, else query groups: k = 128 on bf16 is 6)
                                             (1024, "bf16", 100_003, 128, 50), (768, "f16", 41_000, 100, 30),
                                             (512, "f32", 30_001, 128, 64), (256, "f32", 20_011, 256, 128),
                                             (1024, "bf16", 20_000, 97, 128)])
def test_wide_filter_vs_oracle(native, dim, dtype, n, B, k):
    """65..256 queries at D = 256..1024 take the 128-query FILTER: one workgroup per CU scores every tile once
    for two 64-query groups, the queries streaming through LDS in depth windows.  Fewer tiles than waves (idle
    waves walk the windows on zero-record V#s), a padded second set (B = 129, 80, 97), fp32 rows, row parts
    (k > 16), a mask, deleted rows, ip scores: identical to the oracle and to the same queries 64 at a time.
    The first unmasked search must have launched the 128-query FILTER exactly where the plan takes it."""
    rng = np.random.default_rng(dim + B + n)
    n_parts = (native.kc_for_k(k, dim) + 31) // 32
    # (fp32 rows scan their 16-bit shadow and plan as 16-bit rows; HIPRAG_F32_SHADOW=0 keeps the fp32 plan)
    f32_plan = dtype == "f32" and os.environ.get("HIPRAG_F32_SHADOW", "1") == "0"
    wide_expected = n_parts == 1 or (n_parts <= 7 if f32_plan else (n_parts <= 3 and B <= 128))
    # (raw inner products of the synthetic rows overflow f16 storage: ip on bf16 / fp32 only; fp32 rows reach the
    # MFMA as f16 for cosine, bf16 for ip)
    for metric in ("cosine", "ip") if dtype != "f16" else ("cosine",):
        idx = native.NativeIndex(dim, dtype, metric)
        idx.add_synthetic(9, 0, n)
        raw = R.gen_rows(9, 0, n, dim)
        nq = min(B // 2, n)
        q = np.concatenate([_planted_queries(raw, nq, rng), rng.standard_normal((B - nq, dim)).astype(np.float32)])
        stored = oracle.c_build_synthetic(9, 0, n, dim, dtype, metric)
        qn = R.process_queries(q, metric)
        allowed = rng.random(n) < 0.7
        # 129-256 queries with one row part: the 256-query FILTER (hr_q256.hip) instead
        q256_expected = n_parts == 1 and B > 128
        for m in (None, allowed):
            mk = None if m is None else oracle.mask_from_bool(m)
            w0, x0 = idx.wide_launches(), idx.q256_launches()
            s, r = idx.search(q, k, mk)
            _check(s, r, *oracle.c_search(stored, dtype, qn, k, mk, metric=metric))
            if m is None:
                assert (idx.q256_launches() > x0) == q256_expected
                assert (idx.wide_launches() > w0) == (wide_expected and not q256_expected)
        parts = [idx.search(q[i:i + 64], k) for i in range(0, B, 64)]
        s, r = idx.search(q, k)
        np.testing.assert_array_equal(r, np.concatenate([p[1] for p in parts]))
        if n > 1000:
            gone = np.arange(n // 3, n // 3 + n // 7)
            idx.remove(gone)
            live = np.ones(n, bool)
            live[gone] = False
            s, r = idx.search(q, k)
            _check(s, r, *oracle.c_search(stored, dtype, qn, k, oracle.mask_from_bool(live), metric=metric))
        if n > 500_000:
            break  # (one metric at a million rows)


# ---------------------------------------------------------------- the 256-query FILTER (hr_q256.hip)
@pytest.mark.parametrize("dim,dtype,n,B,k", [(1024, "bf16", 200_003, 256, 10), (768, "bf16", 150_001, 256, 16),
                                             (512, "f16", 100_000, 200, 10), (256, "bf16", 70_001, 129, 5),
                                             (1024, "bf16", 5_000, 256, 10), (1024, "f16", 64, 256, 3),
                                             (768, "bf16", 1_000_003, 256, 10),
                                             # fp32 rows (the store's default dtype): f16 MFMA for cosine, bf16 for
                                             # ip / euclidean; every depth S = 16 / 32 / 48 / 64
                                             (1024, "f32", 100_003, 256, 10), (768, "f32", 50_001, 200, 16),
                                             (512, "f32", 30_011, 256, 10), (256, "f32", 40_009, 129, 5),
                                             (1024, "f32", 3_000, 256, 10), (1024, "f32", 1_000_003, 256, 10)])
def test_q256_filter_vs_oracle(native, dim, dtype, n, B, k):
    """129-256 queries, one row part: ONE launch of the 256-query FILTER scores every tile for four 64-query groups
    (two tiles per wave, query windows through LDS-DMA).  Fewer tiles than one round (5k, 3k and 64 rows: waves on
    zero-record V#s), padded groups (B = 129, 200), 16-bit and fp32 rows, cosine / ip / euclidean, a dense mask,
    deleted rows -- identical to the oracle and to the same batch through two 128-query FILTER launches
    (set_q256(False))."""
    rng = np.random.default_rng(dim + B + n + 1)
    metrics = ("cosine", "ip", "euclidean") if dtype in ("bf16", "f32") and n < 500_000 else ("cosine",)
    for metric in metrics:
        idx = native.NativeIndex(dim, dtype, metric)
        idx.add_synthetic(31, 0, n)
        raw = R.gen_rows(31, 0, n, dim)
        nq = min(B // 2, n)
        q = np.concatenate([_planted_queries(raw, nq, rng), rng.standard_normal((B - nq, dim)).astype(np.float32)])
        stored = oracle.c_build_synthetic(31, 0, n, dim, dtype, metric)
        qn = R.process_queries(q, metric)
        allowed = rng.random(n) < 0.8
        for m in (None, allowed):
            mk = None if m is None else oracle.mask_from_bool(m)
            x0 = idx.q256_launches()
            s, r = idx.search(q, k, mk)
            _check(s, r, *oracle.c_search(stored, dtype, qn, k, mk, metric=metric))
            assert idx.q256_launches() == x0 + 1
        idx.set_q256(False)
        w0, x0 = idx.wide_launches(), idx.q256_launches()
        s2, r2 = idx.search(q, k)
        assert idx.q256_launches() == x0 and idx.wide_launches() == w0 + 2
        idx.set_q256(True)
        s, r = idx.search(q, k)
        np.testing.assert_array_equal(r, r2)
        np.testing.assert_array_equal(s, s2)
        if n > 1000:
            gone = np.arange(n // 4, n // 4 + n // 9)
            idx.remove(gone)
            live = np.ones(n, bool)
            live[gone] = False
            s, r = idx.search(q, k)
            _check(s, r, *oracle.c_search(stored, dtype, qn, k, oracle.mask_from_bool(live), metric=metric))
        idx.close()


def test_q256_filter_periodic_clusters(native):
    """Clusters repeating every 4096 rows (a factor of the 256-query FILTER's wave count): the rotated two-tile
    dealing spreads them, the private regions hold, and the answer is the oracle's."""
    dim, n, B, C = 256, 2_000_000, 256, 4096
    rng = np.random.default_rng(29)
    centers = rng.standard_normal((C, dim)).astype(np.float32)
    centers /= np.linalg.norm(centers, axis=1, keepdims=True)
    noise = R.gen_rows(47, 0, n, dim)
    noise /= np.linalg.norm(noise, axis=1, keepdims=True)
    raw = centers[(np.arange(n, dtype=np.int64) * 2654435761) % C] + 0.7 * noise
    idx = native.NativeIndex(dim, "bf16", "cosine")
    idx.add(raw)
    stored = R.process_rows(raw, "cosine", "bf16")
    q = (raw[rng.choice(n, B, replace=False)] + 0.1 * rng.standard_normal((B, dim))).astype(np.float32)
    before, x0 = idx.stats()["guard_failures"], idx.q256_launches()
    s, r = idx.search(q, 10)
    _check(s, r, *oracle.c_search(stored, "bf16", R.process_queries(q, "cosine"), 10))
    assert idx.q256_launches() == x0 + 1
    assert idx.stats()["guard_failures"] - before <= B // 8


def test_wide_filter_periodic_clusters(native):
    """The 128-query FILTER deals tile pairs round-robin with each full round rotated by a hash of the
    round: clusters repeating every 4096 rows (a factor of the wave count) still reach every wave, so the
    32-slot private regions hold and the guard passes for nearly every query; identical to the oracle."""
    dim, n, B, C = 256, 2_000_000, 128, 4096
    rng = np.random.default_rng(23)
    centers = rng.standard_normal((C, dim)).astype(np.float32)
    centers /= np.linalg.norm(centers, axis=1, keepdims=True)
    noise = R.gen_rows(43, 0, n, dim)
    noise /= np.linalg.norm(noise, axis=1, keepdims=True)
    raw = centers[(np.arange(n, dtype=np.int64) * 2654435761) % C] + 0.7 * noise
    idx = native.NativeIndex(dim, "bf16", "cosine")
    idx.add(raw)
    stored = R.process_rows(raw, "cosine", "bf16")
    q = (raw[rng.choice(n, B, replace=False)] + 0.1 * rng.standard_normal((B, dim))).astype(np.float32)
    before = idx.stats()["guard_failures"]
    s, r = idx.search(q, 10)
    _check(s, r, *oracle.c_search(stored, "bf16", R.process_queries(q, "cosine"), 10))
    assert idx.stats()["guard_failures"] - before <= B // 8


def test_query_groups_pipelined_vs_oracle(native):
    """The bench's pipelined path at B = 256 and 128 (early SAMPLE, two workspaces, dual FILTER
    streams) on a shard large enough for all of them: every batch identical to the oracle."""
    torch = pytest.importorskip("torch")
    from hiprag.dist import ShardedSearch

    dim, n = 128, 1_300_000
    idx = native.NativeIndex(dim, "bf16", "cosine")
    idx.add_synthetic(29, 0, n)
    raw = R.gen_rows(29, 0, n, dim)
    stored = oracle.c_build_synthetic(29, 0, n, dim, "bf16", "cosine")
    rng = np.random.default_rng(12)
    plan = [(256, 10), (128, 100), (256, 10), (64, 10), (256, 32)]
    qs = [np.concatenate([_planted_queries(raw, B // 2, rng), rng.standard_normal((B - B // 2, dim)).astype(np.float32)])
          for B, _ in plan]
    q_dev = [torch.from_numpy(q).cuda() for q in qs]
    outs = [(torch.empty((B, k), dtype=torch.float32, device="cuda"), torch.empty((B, k), dtype=torch.int64, device="cuda"))
            for B, k in plan]
    ready = torch.cuda.Event()
    ready.record()
    ss = ShardedSearch(idx, 0, max_batch=256, max_k=100, device=torch.device("cuda", 0))
    for (B, k), q, (s_o, r_o) in zip(plan, q_dev, outs):
        ss.submit(q, k, s_out=s_o, r_out=r_o, q_ready=ready)
    ss.finalize_all()
    torch.cuda.synchronize()
    for (B, k), q, (s_o, r_o) in zip(plan, qs, outs):
        _check(s_o.cpu().numpy(), r_o.cpu().numpy(), *oracle.c_search(stored, "bf16", R.process_queries(q, "cosine"), k))


def test_async_slots_out_of_order_and_fallback_before_mutation(native):
    """hr_index_search_submit_host / _collect (the store's event-loop path), ADVICE r03:
    (1) two batches in flight are collected in any order and a submit takes whichever slot is free (a third
    while both are busy raises BusyError, so the store takes its worker path);
    (2) a batch whose guard failed (100 duplicates > kc) gets its exact fallback before a remove between
    submit and collect: the answer is the corpus the batch was submitted against, and poll reports state 2
    (ready, needs the fallback) before collect."""
    dim, n = 128, 6000
    raw = R.gen_rows(21, 0, n, dim)
    dups = np.sort(np.random.default_rng(5).choice(n, 100, replace=False))
    raw[dups] = raw[dups[0]]
    idx = native.NativeIndex(dim, "bf16", "cosine")
    idx.add(raw)
    stored = R.process_rows(raw, "cosine", "bf16")
    rng = np.random.default_rng(6)
    qs = [rng.standard_normal((B, dim)).astype(np.float32) for B in (7, 19, 33)]
    refs = [oracle.c_search(stored, "bf16", R.process_queries(q, "cosine"), 10) for q in qs]
    ta = idx.search_submit_host(qs[0], 10)
    tb = idx.search_submit_host(qs[1], 10)
    with pytest.raises(native.BusyError):
        idx.search_submit_host(qs[2], 10)
    _check(*idx.search_collect(tb, 19, 10), *refs[1])
    tc = idx.search_submit_host(qs[2], 10)  # the slot B freed, while A is outstanding
    _check(*idx.search_collect(tc, 33, 10), *refs[2])
    _check(*idx.search_collect(ta, 7, 10), *refs[0])
    # (2) the fallback runs against the rows at submit
    q = np.concatenate([raw[dups[:1]], qs[0][:3]])
    s_ref, r_ref = oracle.c_search(stored, "bf16", R.process_queries(q, "cosine"), 10)
    g0 = idx.stats()["guard_failures"]
    t = idx.search_submit_host(q, 10)
    import time

    for _ in range(2000):
        st = idx.search_poll(t)
        if st:
            break
        time.sleep(0.001)
    assert st == 2
    idx.remove(dups[:5])  # a mutation between submit and collect
    s, r = idx.search_collect(t, len(q), 10)
    _check(s, r, s_ref, r_ref)
    np.testing.assert_array_equal(r[0], dups[:10])
    assert idx.stats()["guard_failures"] > g0
    # and a fresh search sees the removal
    live = np.ones(n, bool)
    live[dups[:5]] = False
    s2, r2 = idx.search(q, 10)
    _check(s2, r2, *oracle.c_search(stored, "bf16", R.process_queries(q, "cosine"), 10, oracle.mask_from_bool(live)))
    idx.close()


def test_every_tile_scanned_exactly_once(native):
    """hr_index_wave_tiles: the tiles each wave of the last k_scan FILTER scanned sum to groups x units -- the
    round-robin dealing (rotated per round), the dynamic tail (600k rows: every wave gets >= 8 static tiles, so the
    last 10 % go out from the counter), row-part teams, query groups and tile lists each visit every unit exactly
    once.  (Results are checked against the oracle elsewhere; this pins the dealing itself.)"""
    n, dim = 600_011, 256
    n_tiles = (n + 31) // 32
    idx = native.NativeIndex(dim, "bf16", "cosine")
    try:
        idx.add_synthetic(4, 0, n)
        rng = np.random.default_rng(1)
        for B, k, groups in ((64, 10, 1), (40, 50, 1), (256, 100, 4)):
            q = rng.standard_normal((B, dim)).astype(np.float32)
            w0 = idx.wide_launches()
            idx.search(q, k)
            assert idx.wide_launches() == w0  # (k_scan, not the 128-query FILTER)
            wt = idx.wave_tiles()
            assert len(wt) % groups == 0 and len(wt) >= groups * 8
            assert int(wt.sum()) == groups * n_tiles, (B, k, int(wt.sum()), groups * n_tiles)
        # tile list: a few documents' contiguous rows -> only their tiles
        sel = np.zeros(n, bool)
        for lo in (1000, 300_000, 599_000):
            sel[lo:lo + 5000] = True
        idx.search(rng.standard_normal((64, dim)).astype(np.float32), 10, oracle.mask_from_bool(sel))
        listed = len(np.unique(np.nonzero(sel)[0] // 32))
        assert int(idx.wave_tiles().sum()) == listed
    finally:
        idx.close()


# ---------------------------------------------------------------- fp32 corpora: the 16-bit scan shadow
@pytest.mark.parametrize("metric", ["cosine", "ip", "l2"])
def test_f32_shadow_incremental_reload_and_off(native, metric, tmp_path, monkeypatch):
    """fp32 rows are streamed by the approximate passes from a 16-bit shadow (hr_internal.hpp rows16), kept current
    lazily: searches between adds (a partial last tile re-converted), removals, a save / load (the shadow rebuilt from
    the loaded rows) and batches of 1 / 40 / 200 queries (k_scan, the 128- and 256-query FILTERs) answer as the
    oracle does, and as an index built with HIPRAG_F32_SHADOW=0 (the fp32 tiles rounded in the kernels)."""
    rng = np.random.default_rng({"cosine": 1, "ip": 2, "l2": 3}[metric])
    dim, n = 512, 12_000
    x = _embedding_like(rng, n, dim, scale=2.0)
    stored = R.process_rows(x, metric, "f32")
    qm = (lambda q: R.process_queries(q, metric)) if metric == "cosine" else (lambda q: q)

    def planted(B, upto):
        j = rng.choice(upto, B, replace=False)
        return (x[j] + 0.05 * rng.standard_normal((B, dim)).astype(np.float32)).astype(np.float32)

    def check(idx, q, k, upto, mask=None):
        s, r = idx.search(q, k, None if mask is None else oracle.mask_from_bool(mask))
        s_ref, r_ref = oracle.c_search(stored[:upto], "f32", qm(q), k,
                                       None if mask is None else oracle.mask_from_bool(mask), metric=metric)
        _check(s, r, s_ref, r_ref)
        return s, r

    monkeypatch.delenv("HIPRAG_F32_SHADOW", raising=False)
    idx = native.NativeIndex(dim, "f32", metric)
    for upto in (5_000, 5_017, n):  # (5,017: the second add lands in the first add's last, partial tile)
        idx.add(x[idx.size()[0]:upto])
        check(idx, planted(40, upto), 10, upto)
    gone = rng.choice(n, 500, replace=False)
    idx.remove(gone)
    allowed = np.ones(n, bool)
    allowed[gone] = False
    results = {}
    for B in (1, 40, 200):
        q = planted(B, n)
        results[B] = (q, check(idx, q, 10, n, allowed))
    p = str(tmp_path / "f32.hri")
    idx.save(p)
    idx2 = native.NativeIndex.load(p, dim=dim, dtype="f32", metric=metric)
    for B, (q, (s, r)) in results.items():
        s2, r2 = idx2.search(q, 10)
        np.testing.assert_array_equal(r2, r)
        np.testing.assert_array_equal(s2, s)
    monkeypatch.setenv("HIPRAG_F32_SHADOW", "0")
    off = native.NativeIndex(dim, "f32", metric)
    off.add(x)
    off.remove(gone)
    for B, (q, (s, r)) in results.items():
        s3, r3 = off.search(q, 10)
        np.testing.assert_array_equal(r3, r)
        np.testing.assert_array_equal(s3, s)

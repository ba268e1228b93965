"""CPU: the oracle is pinned against the golden vectors produced by the reference's own
code (tests/golden/gen_golden.py), and its C and numpy restatements agree bit for bit."""
import hashlib
import json
import os

import numpy as np
import pytest

import oracle
from oracle import ref_numpy as R


def test_c_and_numpy_agree_bitwise():
    rng = np.random.default_rng(0)
    for dim in (1, 63, 64, 100, 128, 257):
        x = R.gen_rows(5, 10, 300, dim)
        assert np.array_equal(oracle.c_gen_rows(5, 10, 300, dim), x)
        xn = R.normalize_rows(x)
        assert np.array_equal(oracle.c_normalize_rows(x).view(np.uint32), xn.view(np.uint32))
        for dt in ("f32", "bf16", "f16"):
            st = R.quantize(xn, dt)
            assert np.array_equal(oracle.c_quantize(xn, dt), st)
            q = R.process_queries(rng.standard_normal((4, dim)).astype(np.float32), "cosine")
            allowed = rng.random(300) < 0.7
            s1, r1 = oracle.c_search(st, dt, q, 7, oracle.mask_from_bool(allowed), row_offset=11)
            s2, r2 = R.search(st, dt, q, 7, allowed, row_offset=11)
            assert np.array_equal(r1, r2) and np.array_equal(s1, s2)


def test_euclidean_c_numpy_and_direct_formula():
    """l2 (euclidean): C and numpy restatements agree bit-for-bit, and the canonical
    1 - ((|q|^2 - 2 q.x) + |x|^2) matches Chroma's similarity 1 - squared distance computed
    directly (chroma_store.py:48-53 hnsw "l2", :135) to fp64 rounding."""
    rng = np.random.default_rng(3)
    for dim in (7, 64, 130):
        x = rng.standard_normal((400, dim)).astype(np.float32)
        for dt in ("f32", "bf16", "f16"):
            st = R.process_rows(x, "l2", dt)
            q = rng.standard_normal((5, dim)).astype(np.float32)
            allowed = rng.random(400) < 0.8
            s1, r1 = oracle.c_search(st, dt, q, 9, oracle.mask_from_bool(allowed), metric="l2")
            s2, r2 = R.search(st, dt, q, 9, allowed, metric="l2")
            assert np.array_equal(r1, r2) and np.array_equal(s1, s2)
            xs = R.dequantize(st, dt).astype(np.float64)
            direct = 1.0 - ((q.astype(np.float64)[:, None, :] - xs[None]) ** 2).sum(-1)
            np.testing.assert_allclose(np.take_along_axis(direct, r1, 1), s1, rtol=0, atol=1e-9 * dim)
            assert np.all(np.diff(s1, axis=1) <= 0)
            pairs = oracle.c_score_pairs(st, dt, q, np.repeat(np.arange(5), 9), r1.reshape(-1), metric="l2")
            assert np.array_equal(pairs.reshape(5, 9), s1)


def test_quantizers_edge_values():
    v = np.array([0.0, -0.0, 1e-40, -1e-40, 6e-8, 3e-8, 2.98e-8, 65504, 65519, 65520, 1e30, -1e30, np.inf, -np.inf,
                  1.0 + 2 ** -8, 1.0 + 3 * 2 ** -9], np.float32)
    assert np.array_equal(oracle.c_quantize(v[None], "f16")[0], R.f32_to_f16(v))
    assert np.array_equal(oracle.c_quantize(v[None], "bf16")[0], R.f32_to_bf16(v))
    assert R.f32_to_bf16(np.array([1.0 + 2 ** -8], np.float32))[0] == 0x3F80  # tie -> even
    assert R.f32_to_bf16(np.array([1.0 + 3 * 2 ** -8], np.float32))[0] == 0x3F82


def test_zero_rows_stay_zero_like_faiss():
    x = np.zeros((2, 70), np.float32)
    x[1, 3] = 5.0
    y = R.normalize_rows(x)
    assert np.all(y[0] == 0) and y[1, 3] == 1.0


def test_c1_golden(golden_dir):
    d = np.load(os.path.join(golden_dir, "c1_retrieval.npz"))
    meta = json.load(open(os.path.join(golden_dir, "c1_retrieval.json")))
    stored = R.process_rows(d["corpus"], "cosine", "f32")
    q = R.process_queries(d["queries"], "cosine")
    s, r = oracle.c_search(stored, "f32", q, 5)
    for b, res in enumerate(meta["results"]["thr0"]):
        assert [f"chunk_{x}" for x in r[b]] == [e["chunk_id"] for e in res]
        assert list(s[b]) == [e["score"] for e in res]  # same canonical fp64 arithmetic: bit-identical
    allowed = np.array([m["group"] == "g1" for m in meta["metas"]])
    s, r = oracle.c_search(stored, "f32", q, 5, oracle.mask_from_bool(allowed))
    for b, res in enumerate(meta["results"]["filtered_g1"]):
        assert [f"chunk_{x}" for x in r[b] if x >= 0] == [e["chunk_id"] for e in res]


def test_ties_golden(golden_dir):
    d = np.load(os.path.join(golden_dir, "ties.npz"))
    meta = json.load(open(os.path.join(golden_dir, "ties.json")))
    corpus = R.gen_rows(7, 0, 20000, 256)
    for s_, dst in zip(d["dup_src"], d["dup_dst"]):
        corpus[dst] = corpus[s_]
    s, r = oracle.c_search(R.process_rows(corpus, "cosine", "f32"), "f32", R.process_queries(d["queries"], "cosine"), 10)
    for b, res in enumerate(meta["results"]):
        assert [f"chunk_{x}" for x in r[b]] == [e["chunk_id"] for e in res]
        assert list(s[b]) == [e["score"] for e in res]
    # planted duplicates really tie and are ordered by row
    top = [e for e in meta["results"][0] if e["score"] == meta["results"][0][0]["score"]]
    rows = [int(e["chunk_id"].split("_")[1]) for e in top]
    assert len(rows) >= 2 and rows == sorted(rows)


def test_corpus_sha256(golden_dir):
    sha = json.load(open(os.path.join(golden_dir, "corpus_sha256.json")))
    for key in ("seed0_rows1000_dim128_bf16_cosine", "seed0_rows1000_dim128_f32_cosine",
                "seed0_rows1000_dim128_bf16_ip", "seed0_rows4096_dim768_f16_cosine"):
        parts = key.split("_")
        n, dim, dt, metric = int(parts[1][4:]), int(parts[2][3:]), parts[3], parts[4]
        st = oracle.c_build_synthetic(0, 0, n, dim, dt, metric, 2)
        assert hashlib.sha256(st.tobytes()).hexdigest() == sha[key]


def test_synthetic_streaming_search_matches_materialised():
    q = R.process_queries(np.random.default_rng(1).standard_normal((3, 96)).astype(np.float32), "cosine")
    st = oracle.c_build_synthetic(4, 50, 2000, 96, "bf16", "cosine", 2)
    s1, r1 = oracle.c_search(st, "bf16", q, 9, row_offset=50)
    s2, r2 = oracle.c_search_synthetic(4, 50, 2000, 96, "bf16", "cosine", q, 9, 2)
    assert np.array_equal(r1, r2) and np.array_equal(s1, s2)


def test_product_generator_matches_oracle():
    """hiprag.synth (bench/query data) uses the same generator the oracle restates."""
    from hiprag import synth

    rows = np.array([0, 5, 99999, 12345678])
    assert np.array_equal(synth.corpus_rows(3, rows, 40), np.stack([R.gen_rows(3, int(r), 1, 40)[0] for r in rows]))


@pytest.mark.parametrize("k", [1, 4, 16])
def test_oracle_k_larger_than_rows(k):
    st = R.process_rows(R.gen_rows(2, 0, 3, 64), "cosine", "bf16")
    s, r = oracle.c_search(st, "bf16", np.ones((1, 64), np.float32), k)
    assert (r[0][: min(k, 3)] >= 0).all() and (r[0][3:] == -1).all()

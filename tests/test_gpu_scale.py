"""GPU parity at the BASELINE.json sizes (configs[1..4]), through the C ABI.

* C3: 10M x 1024 bf16, B = 64 (two batches: planted + isotropic queries), k = 10 and 100, against
  the oracle's exact search over all 10M rows (generated on the fly by the same counter-based
  generator).  Isotropic queries are the worst case for exact-id parity (SURVEY §7 hard part 1:
  top-k gaps shrink with N), so this is where the exactness guard and its collect / exhaustive
  fallbacks must hold; the guard counters (hr_index_stats) are printed.  Also: the pipelined
  two-stream path the bench times, and tombstones + a where-clause bitmap at 10M.
* C2: 1M x 768, f32 and bf16 stores, B = 64, k = 10; the bf16 store's recall@10 against the exact
  answer over the unquantised fp32 rows (the reference's store dtype).
* C5: one 6.25M-row f16 IVF shard (50M / 8), nlist 8192, nprobe 32, k = 100, against the IVF
  restatement (FAISS IndexIVFFlat's algorithm, oracle/ref_numpy.ivf_search) evaluated on the rows
  of the probed lists only.
Bar: ids identical (score desc, row asc), scores equal to the oracle's fp64 canonical scores cast
to fp32 (so within the north_star's 1e-5).
"""
import os

import numpy as np
import pytest

import oracle
from oracle import ref_numpy as R

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def native():
    from hiprag import _native

    _native.load_library()
    assert _native.device_count() >= 1, "no HIP device visible"
    return _native


def _check(s_gpu, r_gpu, s_ref, r_ref):
    np.testing.assert_array_equal(r_gpu, r_ref)
    valid = r_ref >= 0
    np.testing.assert_array_equal(s_gpu[valid], s_ref[valid].astype(np.float32))
    assert np.all(np.isneginf(s_gpu[~valid]))


def _queries(seed, n, dim, B, qseed):
    from hiprag import synth

    planted, _ = synth.planted_queries(seed, n, dim, B, qseed=qseed)
    iso = np.random.default_rng(qseed + 1).standard_normal((B, dim)).astype(np.float32)
    return planted, iso


# ---------------------------------------------------------------- C3: 10M x 1024 bf16
N3, D3, SEED3 = 10_000_000, 1024, 0


@pytest.fixture(scope="module")
def c3(native):
    idx = native.NativeIndex(D3, "bf16", "cosine")
    idx.reserve(N3)
    idx.add_synthetic(SEED3, 0, N3)
    planted, iso = _queries(SEED3, N3, D3, 64, qseed=4242)
    planted2, iso2 = _queries(SEED3, N3, D3, 64, qseed=4343)  # 128 more: the store's 256-query sample
    q = np.concatenate([planted, iso])
    q2 = np.concatenate([planted2, iso2])
    # one oracle pass over the 10M rows for all 256 queries at k = 100; top-10 is its prefix
    s_all, r_all = oracle.c_search_synthetic(SEED3, 0, N3, D3, "bf16", "cosine",
                                             R.process_queries(np.concatenate([q, q2]), "cosine"), 100)
    yield idx, q, s_all[:128], r_all[:128], q2, s_all[128:], r_all[128:]
    idx.close()


@pytest.mark.parametrize("k", [10, 100])
def test_c3_10M_bf16_vs_oracle(c3, k):
    idx, q, s_ref, r_ref, *_ = c3
    before, w0 = idx.stats(), idx.wide_launches()
    # 128 queries in ONE corpus pass: at k = 10 the 128-query FILTER (hr_wide.hip, one launch); at k = 100
    # (kc 160: 5 row parts, more than the 16-bit 128-query FILTER takes) two query groups in one k_scan launch
    s, r = idx.search(q, k)
    after, w1 = idx.stats(), idx.wide_launches()
    print(f"\nC3 10Mx1024 bf16 k={k}: stats {after}, this search: "
          f"guard failures {after['guard_failures'] - before['guard_failures']}, "
          f"exhaustive {after['exhaustive'] - before['exhaustive']}, 128-query FILTER launches {w1 - w0}")
    assert w1 - w0 == (1 if k == 10 else 0)
    # one main pass (stats' main_passes counts FILTER passes; a collect fallback is not one)
    assert after["main_passes"] - before["main_passes"] == 1
    _check(s[:64], r[:64], s_ref[:64, :k], r_ref[:64, :k])    # planted
    _check(s[64:], r[64:], s_ref[64:, :k], r_ref[64:, :k])    # isotropic


def _q256_vs_oracle(fixture, label):
    """The fixture's 256 queries (planted + isotropic, two seeds) in ONE search, asserted to run as one 256-query
    FILTER launch (hr_q256.hip); ids and score bits equal the oracle's over all 10M rows.  Then the same batch with
    the 256-query FILTER off (two 128-query launches) for the A/B, identical again."""
    idx, q, s_ref, r_ref, q2, s2, r2 = fixture
    qq = np.concatenate([q, q2])
    sr, rr = np.concatenate([s_ref, s2])[:, :10], np.concatenate([r_ref, r2])[:, :10]
    for on in (True, False):
        idx.set_q256(on)
        before, w0 = idx.q256_launches(), idx.wide_launches()
        s, r = idx.search(qq, 10)
        after, w1 = idx.q256_launches(), idx.wide_launches()
        print(f"\nC3 {label} B=256 q256={on}: 256-query launches {after - before}, 128-query launches {w1 - w0}, "
              f"stats {idx.stats()}")
        assert after - before == (1 if on else 0)
        assert w1 - w0 == (0 if on else 2)
        _check(s, r, sr, rr)
    idx.set_q256(True)


def test_c3_q256_vs_oracle(c3):
    """the 256-query FILTER at C3 size, explicitly (bf16 rows)."""
    _q256_vs_oracle(c3, "bf16")


def test_c3_pipelined_path_vs_oracle(c3):
    """The bench's path (ShardedSearch: scan + tail streams, early SAMPLE, two workspaces) on the
    same 10M rows: planted and isotropic batches alternate, each identical to the oracle."""
    import torch

    from hiprag.dist import ShardedSearch

    idx, q, s_ref, r_ref, *_ = c3
    k = 10
    qd = torch.from_numpy(q).cuda().view(2, 64, D3)
    ready = torch.cuda.Event()
    ready.record()
    ss = ShardedSearch(idx, 0, max_batch=64, device=torch.device("cuda", 0))
    s_out = torch.empty((4, 64, k), dtype=torch.float32, device="cuda")
    r_out = torch.empty((4, 64, k), dtype=torch.int64, device="cuda")
    for i in range(4):
        ss.submit(qd[i % 2], k, s_out=s_out[i], r_out=r_out[i], q_ready=ready)
    ss.finalize_all()
    torch.cuda.synchronize()
    for i in range(4):
        h = i % 2
        _check(s_out[i].cpu().numpy(), r_out[i].cpu().numpy(), s_ref[64 * h:64 * (h + 1), :k],
               r_ref[64 * h:64 * (h + 1), :k])


# ---------------------------------------------------------------- the reference's own call shapes at C3
# VectorRetriever.retrieve issues ONE query per store search (base_retriever.py:57-63 -> chroma_store.py:118-120);
# a serving process sees many of them at once, which HipVectorStore's micro-batcher coalesces (storage.py).
def _call_shapes(idx, q, s_ref, r_ref):
    """Synchronous searches of B = 1 and B = 16 (the shapes SURVEY §8(d) lists for C3; the second use of a shape
    replays its captured HIP graph), planted and isotropic queries, k = 10 and 100, each identical to the oracle's
    exact answer over all 10M rows."""
    n = 0
    for k in (10, 100):
        for B in (1, 16):
            for h in (0, 64):  # planted, isotropic
                for b0 in range(h, h + 4 * B, B):  # 4 searches of each shape and kind
                    s, r = idx.search(q[b0:b0 + B], k)
                    _check(s, r, s_ref[b0:b0 + B, :k], r_ref[b0:b0 + B, :k])
                    n += 1
    print(f"\n{n} searches of B = 1 / 16: stats {idx.stats()}")


class _LazyTable:
    """Host records of the synthetic collection, computed for the rows a search returns (row r = chunk r % 1000 of
    document r // 1000, the layout tools/bench_async.py loads): the store's _assemble indexes `.a` with the hit rows.
    Building the real 10M-entry tables takes ~95 s of Python, longer than a test may run."""

    def __init__(self, n: int, meta: bool):
        self.n, self.meta, self.a = n, meta, self

    def __len__(self):
        return self.n

    def __getitem__(self, rows):
        rows = np.asarray(rows).reshape(-1)
        out = np.empty(len(rows), object)
        for j, r in enumerate(rows.tolist()):
            d, i = divmod(r, 1000)
            out[j] = {"document_id": f"doc{d}", "chunk_index": i} if self.meta else (f"doc{d}_chunk_{i}", f"doc{d}", "", i)
        return out


class _Count:
    def __init__(self, n):
        self.n = n

    def __len__(self):
        return self.n


def _store_async(idx, dtype, q, s_ref, r_ref, max_batch):
    """256 concurrent single-query ``await store.search(query_embedding=..., top_k=10)`` tasks through HipVectorStore
    over the 10M-row index: the micro-batcher's native launches (hr_index_search_submit_host, eventfd completion,
    hr_index_search_collect, _assemble) -- every answer's chunk ids and score bits equal the oracle's."""
    import asyncio

    from hiprag.rag import HipVectorStore, VectorStoreConfig

    cfg = VectorStoreConfig(backend="hip", collection_name="c3", persist_directory="/tmp/hiprag_c3_store",
                            index_params={"dtype": dtype, "persist": False, "max_batch": max_batch})
    st = HipVectorStore(cfg, index_factory=lambda d: idx)
    st._ensure_index(D3)
    st._records, st._metas, st._id_to_row = _LazyTable(N3, False), _LazyTable(N3, True), _Count(N3)

    async def main():
        return await asyncio.gather(*[st.search(query_embedding=x.tolist(), top_k=10) for x in q])

    try:
        out = asyncio.run(main())
        launches, native = st._batcher.launches, st._batcher.native_launches
    finally:
        st._batcher.close()  # (not st.close(): the index belongs to the module fixture)
    for i, res in enumerate(out):
        want = [f"doc{r // 1000}_chunk_{r % 1000}" for r in r_ref[i, :10].tolist()]
        assert [c.id for c, _ in res] == want, i
        got = np.asarray([sc for _, sc in res], np.float32)
        np.testing.assert_array_equal(got.view(np.uint32), s_ref[i, :10].astype(np.float32).view(np.uint32))
    print(f"\nstore async, max_batch {max_batch}: {launches} launches, {native} through submit_host")
    assert native >= 1 and launches <= -(-len(q) // max_batch) + 2


def test_c3_call_shapes_bf16_vs_oracle(c3):
    idx, q, s_ref, r_ref, *_ = c3
    _call_shapes(idx, q, s_ref, r_ref)


@pytest.mark.parametrize("max_batch", [64, 256])
def test_c3_store_async_256_clients_bf16_vs_oracle(c3, max_batch):
    idx, q, s_ref, r_ref, q2, s2, r2 = c3
    _store_async(idx, "bf16", np.concatenate([q, q2]), np.concatenate([s_ref, s2]), np.concatenate([r_ref, r2]),
                 max_batch)


def test_c3_group_8_shards_pipelined_vs_oracle(c3, native):
    """The single-process multi-GPU handle at C3: one handle striped over 8 shards (on a one-GPU box the
    8 shards share the GPU: dev_ids = [0]*8 -- 8 x 1.25M rows, the per-GPU rows of the 8-GPU node), rows
    generated in place (generator row = handle row, so the corpus is C3's), batches pipelined through
    hr_index_search_submit / _finalize with one host thread per shard: planted and isotropic batches,
    k = 10 and 100, identical to the oracle over all 10M rows."""
    import torch

    _, q, s_ref, r_ref, *_ = c3
    n_vis = native.device_count()
    devs = [i % n_vis for i in range(8)]
    grp = native.NativeIndex(D3, "bf16", "cosine", devices=devs)
    try:
        grp.reserve(N3)
        grp.add_synthetic(SEED3, 0, N3)
        dev = torch.device("cuda", devs[0])
        st = torch.cuda.current_stream(dev).cuda_stream
        qd = torch.from_numpy(q).to(dev).view(2, 64, D3)
        outs = []
        for i, k in enumerate([10, 10, 100, 100, 10, 10]):
            h = i % 2
            s = torch.empty((64, k), dtype=torch.float32, device=dev)
            r = torch.empty((64, k), dtype=torch.int64, device=dev)
            outs.append((grp.search_submit(qd[h].data_ptr(), 64, k, s.data_ptr(), r.data_ptr(), stream=st), h, k, s, r))
        for t, *_ in outs:
            grp.search_finalize(t)
        torch.cuda.synchronize(dev)
        for _, h, k, s, r in outs:
            _check(s.cpu().numpy(), r.cpu().numpy(), s_ref[64 * h:64 * (h + 1), :k], r_ref[64 * h:64 * (h + 1), :k])
        print(f"\nC3 one handle x 8 shards: stats {grp.stats()}, host us {grp.host_us()}")
    finally:
        grp.close()


def test_c3_tombstones_and_filter_vs_oracle(c3):
    """Deleted rows (tombstones) and a where-clause bitmap at 10M: a dense random filter (full scan
    with the mask fused into the scan) and a few documents' contiguous row ranges (tile list)."""
    idx, q, _, _, *_ = c3
    rng = np.random.default_rng(77)
    dead = np.unique(rng.integers(0, N3, 20_000))
    idx.remove(dead)
    live = np.ones(N3, bool)
    live[dead] = False
    dense = rng.random(N3) < 0.5
    docs = np.zeros(N3, bool)
    for lo in (123_456, 5_000_000, 9_990_000):
        docs[lo:lo + 10_000] = True
    qp = q[:64]
    qn = R.process_queries(qp, "cosine")
    try:
        for allowed in (None, dense, docs):
            m = live if allowed is None else (live & allowed)
            k = 10
            s, r = idx.search(qp, k, None if allowed is None else oracle.mask_from_bool(allowed))
            s_ref, r_ref = oracle.c_search_synthetic(SEED3, 0, N3, D3, "bf16", "cosine", qn, k,
                                                     mask=oracle.mask_from_bool(m))
            _check(s, r, s_ref, r_ref)
    finally:
        print(f"\nC3 filtered: stats {idx.stats()}")


# ---------------------------------------------------------------- C3 on the store's default dtype: fp32 rows
@pytest.fixture(scope="module")
def c3_f32(native):
    idx = native.NativeIndex(D3, "f32", "cosine")
    idx.reserve(N3)
    idx.add_synthetic(SEED3, 0, N3)
    planted, iso = _queries(SEED3, N3, D3, 64, qseed=5151)
    planted2, iso2 = _queries(SEED3, N3, D3, 64, qseed=5252)
    q = np.concatenate([planted, iso])
    q2 = np.concatenate([planted2, iso2])
    s_all, r_all = oracle.c_search_synthetic(SEED3, 0, N3, D3, "f32", "cosine",
                                             R.process_queries(np.concatenate([q, q2]), "cosine"), 100)
    yield idx, q, s_all[:128], r_all[:128], q2, s_all[128:], r_all[128:]
    idx.close()


@pytest.mark.parametrize("k", [10, 100])
def test_c3_10M_f32_vs_oracle(c3_f32, k):
    """The drop-in store's default dtype (fp32 rows, the reference's: faiss_store.py:98, :148-154; Chroma
    float32) at the headline size, 40.96 GB: fp32 rows reach the MFMA as f16 and rely on the exactness guard,
    whose window is widest here (isotropic queries over 10M rows).  B = 64 runs k_scan; B = 128 the fp32
    128-query FILTER where the plan takes it (asserted through hr_index_wide_launches).  Identical to the oracle's
    exact fp32 answer; the guard counters are printed."""
    from hiprag import _native

    idx, q, s_ref, r_ref, *_ = c3_f32
    # the 128-query FILTER takes up to 3 row parts on 16-bit rows -- fp32 rows scan their 16-bit shadow and plan
    # alike -- and up to 7 on fp32 rows streamed as such (HIPRAG_F32_SHADOW=0)
    n_parts = (_native.kc_for_k(k, 1024) + 31) // 32
    wide_ok = n_parts <= (7 if os.environ.get("HIPRAG_F32_SHADOW", "1") == "0" else 3)
    for B in (64, 128):
        before, w0 = idx.stats(), idx.wide_launches()
        if B == 64:
            outs = [idx.search(q[:64], k), idx.search(q[64:], k)]
            s, r = np.concatenate([o[0] for o in outs]), np.concatenate([o[1] for o in outs])
        else:
            s, r = idx.search(q, k)
        after, w1 = idx.stats(), idx.wide_launches()
        print(f"\nC3 10Mx1024 f32 k={k} B={B}: 128-query FILTER launches {w1 - w0}, guard failures "
              f"{after['guard_failures'] - before['guard_failures']}, exhaustive {after['exhaustive'] - before['exhaustive']}")
        assert (w1 - w0 > 0) == (B == 128 and wide_ok)
        _check(s[:64], r[:64], s_ref[:64, :k], r_ref[:64, :k])    # planted
        _check(s[64:], r[64:], s_ref[64:, :k], r_ref[64:, :k])    # isotropic


def test_c3_f32_q256_vs_oracle(c3_f32):
    """VERDICT r05 missing #2: the 256-query FILTER on fp32 rows (the drop-in store's default dtype, faiss_store.py:98)
    at C3 size -- one corpus pass for 256 queries instead of two -- identical to the oracle's exact fp32 answer."""
    _q256_vs_oracle(c3_f32, "f32")


def test_c3_call_shapes_f32_vs_oracle(c3_f32):
    idx, q, s_ref, r_ref, *_ = c3_f32
    _call_shapes(idx, q, s_ref, r_ref)


@pytest.mark.parametrize("max_batch", [64, 256])
def test_c3_store_async_256_clients_f32_vs_oracle(c3_f32, max_batch):
    idx, q, s_ref, r_ref, q2, s2, r2 = c3_f32
    _store_async(idx, "f32", np.concatenate([q, q2]), np.concatenate([s_ref, s2]), np.concatenate([r_ref, r2]),
                 max_batch)


# ---------------------------------------------------------------- C2: 1M x 768, f32 and bf16
@pytest.mark.parametrize("dtype", ["f32", "bf16"])
def test_c2_1M_768_vs_oracle(native, dtype):
    n, dim, seed = 1_000_000, 768, 11
    idx = native.NativeIndex(dim, dtype, "cosine")
    try:
        idx.add_synthetic(seed, 0, n)
        planted, iso = _queries(seed, n, dim, 64, qseed=99)
        q = np.concatenate([planted, iso])
        s, r = idx.search(q, 10)
        s_ref, r_ref = oracle.c_search_synthetic(seed, 0, n, dim, dtype, "cosine", R.process_queries(q, "cosine"), 10)
        print(f"\nC2 1Mx768 {dtype}: stats {idx.stats()}")
        _check(s, r, s_ref, r_ref)
    finally:
        idx.close()


def test_c2_bf16_store_recall_vs_fp32(native):
    """How far the bf16 store departs from the reference's answers: the reference stores fp32
    (faiss_store.py:98 normalize_L2 + IndexFlatIP over float32; Chroma float32), so its exact answer
    is the top-10 over the UNQUANTISED rows.  The bf16 store is exact over its stored values (the
    test above); against the fp32 answer it differs where two rows' scores lie closer than the bf16
    rounding of their dot products.  Measured recall@10 is printed and bounded (planted queries: one
    clear neighbour + background ranks; isotropic: every rank in the dense tail).  The f32 store is
    identical to the fp32 answer (test_c2_1M_768_vs_oracle[f32])."""
    n, dim, seed = 1_000_000, 768, 11
    idx = native.NativeIndex(dim, "bf16", "cosine")
    try:
        idx.add_synthetic(seed, 0, n)
        planted, iso = _queries(seed, n, dim, 64, qseed=99)
        q = np.concatenate([planted, iso])
        _, r = idx.search(q, 10)
        _, r32 = oracle.c_search_synthetic(seed, 0, n, dim, "f32", "cosine", R.process_queries(q, "cosine"), 10)
        rec = [np.mean([len(set(r[i]) & set(r32[i])) / 10 for i in sl]) for sl in (range(64), range(64, 128))]
        top1 = float(np.mean(r[:, 0] == r32[:, 0]))
        print(f"\nC2 1Mx768 bf16 store vs exact fp32: recall@10 planted {rec[0]:.4f} isotropic {rec[1]:.4f}, "
              f"top-1 agreement {top1:.4f}")
        assert top1 == 1.0
        assert rec[0] >= 0.95 and rec[1] >= 0.95
    finally:
        idx.close()


# ---------------------------------------------------------------- C5: one 6.25M f16 IVF shard
def test_c5_ivf_6p25M_shard_vs_oracle(native):
    """nlist 8192, nprobe 32, k = 100 over the 6.25M rows one of 8 GPUs holds of the 50M corpus.
    The oracle restates IndexIVFFlat: exact coarse scores of every centroid (canonical fp64 over the
    index's fp32 centroids), the nprobe best lists (score desc, list asc), then the exact top-k of
    the rows of those lists (score desc, id asc) -- evaluated here on those rows only."""
    import torch

    from hiprag import synth
    from hiprag.ivf import IvfIndex

    n, dim, nlist, nprobe, k, seed, row0 = 6_250_000, 1024, 8192, 32, 100, 5, 12_500_000
    ivf = IvfIndex(dim, nlist, dtype="f16")
    try:
        sample = torch.empty((nlist * 16, dim), dtype=torch.float32, device="cuda")
        native.gen_rows_device(seed, row0, nlist * 16, dim, sample.data_ptr(),
                               torch.cuda.current_stream().cuda_stream)
        ivf.train(sample, iters=4, seed=0)
        del sample
        ivf.build_synthetic(seed, row0, n)
        rng = np.random.default_rng(7)
        x = synth.corpus_rows(seed, row0 + rng.choice(n, 8, replace=False), dim)
        eps = rng.standard_normal(x.shape).astype(np.float32)
        planted = x / np.linalg.norm(x, axis=1, keepdims=True) + 0.05 * eps / np.linalg.norm(eps, axis=1, keepdims=True)
        iso = rng.standard_normal((8, dim)).astype(np.float32)
        q = np.concatenate([planted, iso]).astype(np.float32)
        B = len(q)
        qd = torch.from_numpy(q).cuda()
        cand = torch.empty((B, k, 2), dtype=torch.float64, device="cuda")
        bound = torch.empty(B, dtype=torch.float64, device="cuda")
        probes = torch.empty((B, nprobe, 2), dtype=torch.float64, device="cuda")
        ivf.search_candidates(qd, k, nprobe, cand, bound, probes=probes)
        torch.cuda.synchronize()
        got_probe = probes.view(torch.int64)[..., 1].cpu().numpy()
        got_ids = cand.view(torch.int64)[..., 1].cpu().numpy()
        got_s = cand[..., 0].cpu().numpy()
        # coarse stage: canonical fp64 scores of every centroid
        qn = R.process_queries(q, "cosine")
        cent = ivf.centroids[:, :dim].cpu().numpy()
        lists = np.arange(nlist)
        members = ivf.list_members()
        for b in range(B):
            coarse = R.canon_sum(qn[b].astype(np.float64)[None, :] * cent.astype(np.float64))
            p_ref = lists[np.lexsort((lists, -coarse))][:nprobe]
            np.testing.assert_array_equal(got_probe[b], p_ref)
            ids = np.sort(np.concatenate([members[l] for l in p_ref]))
            stored = R.process_rows(synth.corpus_rows(seed, ids, dim), "cosine", "f16")
            s_ref, r_ref = oracle.c_search(stored, "f16", qn[b:b + 1], k)
            ok = r_ref[0] >= 0
            np.testing.assert_array_equal(got_ids[b][ok], ids[r_ref[0][ok]])
            assert np.all(got_ids[b][~ok] == -1)
            np.testing.assert_array_equal(got_s[b][ok], s_ref[0][ok])
        assert torch.all(torch.isneginf(bound))
    finally:
        ivf.close()


# ---------------------------------------------------------------- C4: 100k-chunk ingest -> query
def test_c4_100k_chunk_ingest_then_retrieve(tmp_path):
    """BASELINE configs[3]: split -> in-process embed -> hr_index_add_device for 100k chunks, then
    queries through the reference retriever API.  Stored rows are bit-equal to the oracle's bf16
    quantisation of the vectors the embedder produced; retrieval ids are identical to the oracle's
    exact search over them; re-ingesting a document replaces its chunks (processors.py:364-418)."""
    import asyncio
    import time

    import torch

    from hiprag.rag import BatchedVectorRetriever, ChunkingConfig, Document, HipVectorStore, RetrieverConfig, \
        VectorStoreConfig
    from hiprag.rag.ingest import GpuIngestor
    from hiprag.rag.rocm_embedder import TorchRocmEmbedder

    emb = TorchRocmEmbedder(preset="tiny", batch_size=512, max_length=64, seed=2)
    cfg = VectorStoreConfig(backend="hip", collection_name="kb100k", persist_directory=str(tmp_path),
                            index_params={"dtype": "bf16", "persist": True})
    store = HipVectorStore(cfg)
    ing = GpuIngestor(store, emb, chunking=ChunkingConfig(chunk_size=200, chunk_overlap=20), summary_index=False)
    seen = []
    inner = emb.embed_texts_device
    emb.embed_texts_device = lambda texts: seen.append(inner(texts)) or seen[-1]
    rng = np.random.default_rng(3)
    words = np.array([f"t{i}" for i in range(5000)])
    n_docs, sents = 2000, 260  # ~54 chunks of <= 200 chars per document
    docs = [Document(id=f"d{d}", content=". ".join(" ".join(rng.choice(words, 6)) for _ in range(sents)),
                     metadata={"source": f"s{d % 17}"}) for d in range(n_docs)]
    t0 = time.time()
    n = asyncio.run(ing.ingest(docs))
    print(f"\nC4 ingest: {n} chunks in {time.time() - t0:.1f}s")
    assert n >= 100_000 and asyncio.run(store.count()) == n
    vecs = torch.cat(seen).cpu().numpy()
    assert len(vecs) == n
    stored = store._index.get_rows(np.arange(n))
    expect = R.process_rows(vecs, "cosine", "bf16")
    np.testing.assert_array_equal(stored, R.dequantize(expect, "bf16"))
    ids = [r[0] for r in store._records]
    queries = [" ".join(rng.choice(words, 5)) for _ in range(16)]
    retr = BatchedVectorRetriever(store, emb, RetrieverConfig(top_k=10, similarity_threshold=0.0))
    got = asyncio.run(retr.batch_retrieve(queries, top_k=10))
    qv = R.process_queries(emb.encode_queries(queries).cpu().numpy(), "cosine")
    s_ref, r_ref = oracle.c_search(expect, "bf16", qv, 10)
    assert [[x.chunk.id for x in res] for res in got] == [[ids[j] for j in rr] for rr in r_ref]
    for res, sr in zip(got, s_ref):
        np.testing.assert_array_equal(np.float32([x.score for x in res]), sr.astype(np.float32))
    # re-ingest one document: its old chunks are tombstoned, the new ones appended
    new = Document(id="d5", content="completely different text about t1 t2 t3. " * 20, metadata={"source": "new"})
    old_rows = [store._id_to_row[i] for i in ids if i.startswith("d5_chunk_")]
    n_new = asyncio.run(ing.chunk_and_store(new))
    assert asyncio.run(store.count()) == n - len(old_rows) + n_new
    allowed = np.ones(n, bool)
    allowed[old_rows] = False
    vec_new = seen[-1].cpu().numpy()
    all_stored = np.concatenate([expect, R.process_rows(vec_new, "cosine", "bf16")])
    allowed = np.concatenate([allowed, np.ones(len(vec_new), bool)])
    got2 = asyncio.run(retr.batch_retrieve(queries[:4], top_k=10))
    s2, r2 = oracle.c_search(all_stored, "bf16", qv[:4], 10, oracle.mask_from_bool(allowed))
    ids2 = [r[0] if r is not None else None for r in store._records]
    assert [[x.chunk.id for x in res] for res in got2] == [[ids2[j] for j in rr] for rr in r2]

"""GPU: multi-device index handles (hr_index_create with n_dev > 1, hr_group.hip) behind the drop-in
store -- one handle whose rows are striped over several shards, each on its own stream/device, the
candidates gathered to the primary device and merged.  With one visible GPU the shards share it
(dev_ids = [0, 0, ...]): the same striping, per-shard kernels, peer-copy gather and merge run.
Bar: identical to the CPU oracle AND to a single-device index holding the same rows (ids, scores,
tie order), through every path -- scan + guard, collect fallback, exhaustive (k > HR_MAX_K),
masks / tile lists, tombstones, incremental adds, save / load across device counts, device queries."""
import asyncio

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


def _devs(G):
    from hiprag import _native

    n = _native.device_count()
    return [i % n for i in range(G)]


def _check(s_gpu, r_gpu, s_ref, r_ref):
    np.testing.assert_array_equal(r_gpu, r_ref)
    valid = r_ref >= 0
    np.testing.assert_array_equal(s_gpu[valid], s_ref[valid].astype(np.float32))
    assert np.all(np.isneginf(s_gpu[~valid]))


def _queries(raw, B, rng):
    n, dim = raw.shape
    j = rng.choice(n, B // 2, replace=False)
    base = raw[j] / np.linalg.norm(raw[j], axis=1, keepdims=True)
    planted = base + 0.05 * rng.standard_normal((len(j), dim)).astype(np.float32) / np.sqrt(dim)
    return np.concatenate([planted, rng.standard_normal((B - len(j), dim))]).astype(np.float32)


@pytest.mark.parametrize("G,dtype,metric", [(2, "bf16", "cosine"), (3, "f16", "cosine"), (2, "f32", "l2"),
                                            (4, "bf16", "ip")])
def test_group_matches_oracle_and_single(native, G, dtype, metric):
    rng = np.random.default_rng(G * 7)
    dim, n = 256, 40_017  # not a multiple of 32 * G: partial last tiles
    raw = R.gen_rows(13, 0, n, dim)
    grp = native.NativeIndex(dim, dtype, metric, devices=_devs(G))
    one = native.NativeIndex(dim, dtype, metric)
    for lo, hi in [(0, 7), (7, 20_000), (20_000, 20_033), (20_033, n)]:  # incremental, ragged adds
        assert grp.add(raw[lo:hi]) == lo
        one.add(raw[lo:hi])
    assert grp.size() == one.size() == (n, n)
    np.testing.assert_array_equal(grp.get_rows([0, 31, 32, 33, 64 * G + 5, n - 1]),
                                  one.get_rows([0, 31, 32, 33, 64 * G + 5, n - 1]))
    gone = rng.choice(n, 900, replace=False)
    grp.remove(gone)
    one.remove(gone)
    assert grp.size() == (n, n - 900)
    q = _queries(raw, 64, rng)
    stored = R.process_rows(raw, metric, dtype)
    qn = R.process_queries(q, metric)
    live = ~np.isin(np.arange(n), gone)
    allowed = rng.random(n) < 0.5
    docs = np.zeros(n, bool)
    docs[1000:1500] = docs[30_000:30_100] = True
    for k in (10, 100):
        for m in (None, allowed, docs):
            mk = None if m is None else oracle.mask_from_bool(m)
            s, r = grp.search(q, k, mk)
            s_ref, r_ref = oracle.c_search(stored, dtype, qn, k, oracle.mask_from_bool(live if m is None else live & m),
                                           metric=metric)
            _check(s, r, s_ref, r_ref)
            s1, r1 = one.search(q, k, mk)
            np.testing.assert_array_equal(r, r1)
            np.testing.assert_array_equal(s, s1)
    grp.close()
    one.close()


def test_group_fallbacks_and_exhaustive(native):
    """Planted duplicates spread over every shard force the guard's collect fallback; concentrated
    rows overflow the collect window into the exhaustive pass; k > HR_MAX_K takes the exhaustive
    path on every shard with a host merge -- all identical to the oracle."""
    dim, n, G = 128, 9000, 3
    raw = R.gen_rows(9, 0, n, dim)
    dups = np.sort(np.random.default_rng(2).choice(n, 150, replace=False))
    raw[dups] = raw[dups[0]]
    grp = native.NativeIndex(dim, "bf16", "cosine", devices=_devs(G))
    grp.add(raw)
    q = np.concatenate([raw[dups[:1]], R.gen_rows(99, 0, 3, dim)]).astype(np.float32)
    stored = R.process_rows(raw, "cosine", "bf16")
    qn = R.process_queries(q, "cosine")
    before = grp.stats()
    for k in (10, 100, native.HR_MAX_K + 40):
        s, r = grp.search(q, k)
        _check(s, r, *oracle.c_search(stored, "bf16", qn, k))
    assert grp.stats()["guard_failures"] > before["guard_failures"]
    assert grp.stats()["exhaustive"] > 0
    np.testing.assert_array_equal(grp.search(q[:1], 10)[1][0], dups[:10])
    rng = np.random.default_rng(21)
    base = rng.standard_normal(dim).astype(np.float32)
    conc = (base + 1e-4 * rng.standard_normal((6000, dim))).astype(np.float32)
    g2 = native.NativeIndex(dim, "f16", "cosine", devices=_devs(2))
    g2.add(conc)
    qc = np.stack([conc[5], base]).astype(np.float32)
    _check(*g2.search(qc, 10), *oracle.c_search(R.process_rows(conc, "cosine", "f16"), "f16",
                                                R.process_queries(qc, "cosine"), 10))
    grp.close()
    g2.close()


def test_group_synthetic_save_load_across_device_counts(native, tmp_path):
    """add_synthetic stripes the generator rows; a group's file is the single-index layout, so it
    loads into one device and a single index's file loads into a group -- same answers."""
    dim, n = 384, 70_001
    grp = native.NativeIndex(dim, "bf16", "cosine", devices=_devs(2))
    grp.reserve(n)
    grp.add_synthetic(31, 0, 50_000)
    grp.add_synthetic(31, 50_000, n - 50_000)
    grp.remove([5, 40, 69_999])
    raw = R.gen_rows(31, 0, n, dim)
    rng = np.random.default_rng(3)
    q = _queries(raw, 40, rng)
    live = np.ones(n, bool)
    live[[5, 40, 69_999]] = False
    ref = oracle.c_search_synthetic(31, 0, n, dim, "bf16", "cosine", R.process_queries(q, "cosine"), 20,
                                    mask=oracle.mask_from_bool(live))
    _check(*grp.search(q, 20), *ref)
    p = str(tmp_path / "g.hri")
    grp.save(p)
    one = native.NativeIndex.load(p)
    assert one.size() == (n, n - 3)
    _check(*one.search(q, 20), *ref)
    p1 = str(tmp_path / "one.hri")
    one.save(p1)
    g3 = native.NativeIndex.load(p1, devices=_devs(3))
    assert g3.size() == (n, n - 3)
    _check(*g3.search(q, 20), *ref)
    np.testing.assert_array_equal(g3.get_rows(np.arange(0, n, 997)), one.get_rows(np.arange(0, n, 997)))
    for x in (grp, one, g3):
        x.close()


def test_group_device_queries_and_store(native, tmp_path):
    """hr_index_search_device on a group (queries + outputs on the primary device, device mask) and
    the drop-in store with index_params.devices: results identical to a single-device store."""
    import torch

    from hiprag.rag import Chunk, HipVectorStore, VectorStoreConfig

    dim, n = 128, 20_000
    raw = R.gen_rows(17, 0, n, dim)
    grp = native.NativeIndex(dim, "bf16", "cosine", devices=_devs(2))
    grp.add(raw)
    rng = np.random.default_rng(5)
    q = _queries(raw, 33, rng)
    allowed = rng.random(n) < 0.3
    qd = torch.from_numpy(q).cuda()
    md = torch.from_numpy(oracle.mask_from_bool(allowed).view(np.int64)).cuda()
    s = torch.empty((33, 10), dtype=torch.float32, device="cuda")
    r = torch.empty((33, 10), dtype=torch.int64, device="cuda")
    grp.search_device(qd.data_ptr(), 33, 10, s.data_ptr(), r.data_ptr(), mask_ptr=md.data_ptr(),
                      stream=torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    ref = oracle.c_search(R.process_rows(raw, "cosine", "bf16"), "bf16", R.process_queries(q, "cosine"), 10,
                          oracle.mask_from_bool(allowed))
    _check(s.cpu().numpy(), r.cpu().numpy(), *ref)
    grp.close()

    def store(devs, name):
        cfg = VectorStoreConfig(backend="hip", collection_name=name, persist_directory=str(tmp_path),
                                index_params={"dtype": "bf16", "devices": devs, "fsync": False})
        return HipVectorStore(cfg)

    chunks = [Chunk(id=f"c{i}", document_id=f"d{i // 50}", content=str(i), chunk_index=i % 50,
                    metadata={"src": f"s{i % 7}"}, embedding=raw[i].tolist()) for i in range(3000)]
    a, b = store(_devs(2), "multi"), store([0], "single")
    for st in (a, b):
        asyncio.run(st.add_chunks(chunks[:1000]))
        asyncio.run(st.add_chunks(chunks[1000:]))
        asyncio.run(st.delete_by_document_id("d3"))
    for f in (None, {"src": "s2"}):
        ra = a.search_batch(q[:8], 7, f)
        rb = b.search_batch(q[:8], 7, f)
        assert [[(c.id, sc) for c, sc in x] for x in ra] == [[(c.id, sc) for c, sc in x] for x in rb]
    a.close()
    a2 = store(_devs(2), "multi")  # reload: snapshot + journal on the group
    assert asyncio.run(a2.count()) == 2950
    ra = a2.search_batch(q[:8], 7)
    rb = b.search_batch(q[:8], 7)
    assert [[c.id for c, _ in x] for x in ra] == [[c.id for c, _ in x] for x in rb]


def test_group_pipelined_submit_finalize(native):
    """hr_index_search_submit / _finalize on a group handle: batches of different sizes in flight two at a
    time (one host thread per shard), one of them forcing the guard's collect fallback (planted duplicates
    on every shard), finalized in and out of order, a synchronous search and an add between submits
    (they finalize what is in flight) -- every batch identical to the oracle."""
    import torch

    dim, n, G = 128, 30_000, 3
    raw = R.gen_rows(41, 0, n, dim)
    dups = np.sort(np.random.default_rng(4).choice(n, 150, replace=False))
    raw[dups] = raw[dups[0]]
    grp = native.NativeIndex(dim, "bf16", "cosine", devices=_devs(G))
    grp.add(raw[:20_000])
    rng = np.random.default_rng(8)
    dev = torch.device("cuda", _devs(1)[0])
    st = torch.cuda.current_stream(dev).cuda_stream

    def ref(rows_n, q, k):
        return oracle.c_search(R.process_rows(raw[:rows_n], "cosine", "bf16"), "bf16", R.process_queries(q, "cosine"), k)

    batches = []
    for i, (B, k) in enumerate([(64, 10), (17, 10), (33, 100), (64, 10), (5, 3)]):
        q = _queries(raw[:20_000], B, rng)
        if i == 2:
            q[0] = raw[dups[0]]  # a duplicated row: exact ties across shards -> collect fallback
        qd = torch.from_numpy(q).to(dev)
        s = torch.full((B, k), 7.0, dtype=torch.float32, device=dev)
        r = torch.full((B, k), 7, dtype=torch.int64, device=dev)
        t = grp.search_submit(qd.data_ptr(), B, k, s.data_ptr(), r.data_ptr(), stream=st)
        assert t > 0
        batches.append((t, q, qd, s, r, k))
    before = grp.stats()["guard_failures"]
    grp.search_finalize(batches[4][0])   # newest first: the older ones were finalized by later submits
    grp.search_finalize(batches[3][0])
    grp.search_finalize(batches[3][0])   # twice: no-op
    torch.cuda.synchronize(dev)
    for t, q, qd, s, r, k in batches:
        _check(s.cpu().numpy(), r.cpu().numpy(), *ref(20_000, q, k))
    assert grp.stats()["guard_failures"] >= before
    # a submit, then an add and a synchronous search before its finalize
    q = _queries(raw[:20_000], 40, rng)
    qd = torch.from_numpy(q).to(dev)
    s = torch.empty((40, 10), dtype=torch.float32, device=dev)
    r = torch.empty((40, 10), dtype=torch.int64, device=dev)
    t = grp.search_submit(qd.data_ptr(), 40, 10, s.data_ptr(), r.data_ptr(), stream=st)
    grp.add(raw[20_000:])
    _check(s.cpu().numpy(), r.cpu().numpy(), *ref(20_000, q, 10))   # final before the add ran
    _check(*grp.search(q, 10), *ref(n, q, 10))
    grp.search_finalize(t)
    h = grp.host_us()
    assert h["batches"] == 6 and h["submit_us"] > 0 and h["shard_thread_us"] > 0
    grp.close()

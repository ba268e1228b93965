"""CPU: host logic of HipVectorStore that round 1 left O(N) -- incremental crash-safe persistence,
the predicate-cached where-clause compiler, the search micro-batcher, raw-embedding fidelity.
The device index is the oracle-backed tests/fake_index.OracleIndex (host-logic tests only)."""
import asyncio
import json
import os

import numpy as np
import pytest

from fake_index import AsyncOracleIndex, OracleIndex
from hiprag.rag import Chunk, HipVectorStore, RetrieverConfig, VectorRetriever, VectorStoreConfig
from hiprag.rag import filters as F
from hiprag.rag import persist as P


def run(coro):
    return asyncio.run(coro)


def make_store(tmp_path, dtype="f32", **params):
    cfg = VectorStoreConfig(backend="hip", collection_name="kb", persist_directory=str(tmp_path),
                            index_params={"dtype": dtype, "persist": True, "fsync": False, **params})
    return HipVectorStore(cfg, index_factory=lambda dim: OracleIndex(dim, dtype),
                          index_loader=lambda path, dim, dt, metric: OracleIndex.load(path))


def chunks(doc, n, dim=16, seed=0, start=0):
    rng = np.random.default_rng(seed)
    return [Chunk(id=f"{doc}_chunk_{i}", document_id=doc, content=f"{doc} {i}", chunk_index=i,
                  metadata={"source": f"src_{doc}", "index_type": "index_content"},
                  embedding=rng.standard_normal(dim).astype(np.float32).tolist()) for i in range(start, start + n)]


def files(tmp_path):
    return {f: os.path.getsize(os.path.join(tmp_path, f)) for f in os.listdir(tmp_path)}


def test_journal_writes_o_chunk_bytes_and_replays(tmp_path):
    s = make_store(tmp_path)
    run(s.add_chunks(chunks("d0", 200)))          # first write: generation-1 snapshot
    f1 = files(tmp_path)
    assert "kb.manifest.json" in f1 and "kb.g1.hri" in f1
    run(s.add_chunks(chunks("d1", 10, seed=1)))   # later writes: journal only
    run(s.add_chunks(chunks("d2", 10, seed=2)))
    run(s.delete_by_document_id("d0"))
    f2 = files(tmp_path)
    assert f2["kb.g1.hri"] == f1["kb.g1.hri"]     # snapshot untouched
    # two adds of 10 rows x 16 dims + records + one delete of 200 rows: a few KB, not a rewrite
    assert f2["kb.g1.journal"] < 20_000
    q = np.random.default_rng(9).standard_normal((3, 16)).astype(np.float32)
    want = [[(c.id, sc) for c, sc in r] for r in s.search_batch(q, 5)]
    s2 = make_store(tmp_path)                      # reload = snapshot + journal replay
    assert run(s2.count()) == run(s.count()) == 20
    assert [[(c.id, sc) for c, sc in r] for r in s2.search_batch(q, 5)] == want
    assert run(s2.get_by_id("d0_chunk_3")) is None and run(s2.get_by_id("d1_chunk_3")) is not None


def test_torn_journal_tail_is_dropped(tmp_path):
    s = make_store(tmp_path)
    run(s.add_chunks(chunks("d0", 5)))
    run(s.add_chunks(chunks("d1", 5, seed=1)))
    run(s.add_chunks(chunks("d2", 5, seed=2)))
    j = os.path.join(tmp_path, "kb.g1.journal")
    data = open(j, "rb").read()
    with open(j, "wb") as f:  # a crash in the middle of the last append
        f.write(data[:-7])
    s2 = make_store(tmp_path)
    assert run(s2.count()) == 10 and run(s2.get_by_id("d2_chunk_0")) is None
    assert os.path.getsize(j) < len(data) - 7  # truncated to the last complete entry
    run(s2.add_chunks(chunks("d3", 2, seed=3)))  # and appends continue from there
    assert run(make_store(tmp_path).count()) == 12


def test_flush_compacts_and_a_crash_mid_flush_keeps_the_old_generation(tmp_path):
    s = make_store(tmp_path)
    run(s.add_chunks(chunks("d0", 20)))
    run(s.add_chunks(chunks("d1", 20, seed=1)))
    s.flush()
    f = files(tmp_path)
    assert "kb.g2.hri" in f and "kb.g1.hri" not in f and "kb.g1.journal" not in f
    assert json.load(open(os.path.join(tmp_path, "kb.manifest.json")))["gen"] == 2
    # a crash after the next generation's data files but before its manifest: the old one is served
    s._index.save(os.path.join(tmp_path, "kb.g3.hri"))
    assert run(make_store(tmp_path).count()) == 40


def test_row_count_mismatch_refuses_and_header_wins(tmp_path):
    s = make_store(tmp_path, dtype="bf16")
    run(s.add_chunks(chunks("d0", 8)))
    # the files' dtype / metric win over the config's
    s2 = make_store(tmp_path, dtype="f32")
    assert s2.dtype == "bf16"
    rows = os.path.join(tmp_path, "kb.g1.rows.jsonl")
    lines = open(rows).read().splitlines()
    with open(rows, "w") as f:
        f.write("\n".join(lines[:-1]) + "\n")  # one record lost
    with pytest.raises(RuntimeError):
        make_store(tmp_path)


def test_deferred_block_writes_one_snapshot(tmp_path):
    s = make_store(tmp_path)
    run(s.add_chunks(chunks("d0", 4)))
    with s.deferred_save():
        for d in range(1, 6):
            run(s.delete_by_document_id(f"d{d - 1}"))
            run(s.add_chunks(chunks(f"d{d}", 4, seed=d)))
    f = files(tmp_path)
    assert "kb.g2.hri" in f and not any(k.endswith(".journal") for k in f)
    assert run(make_store(tmp_path).count()) == 4


def test_keep_embeddings_returns_the_raw_fp32_vector(tmp_path):
    s = make_store(tmp_path, dtype="bf16", keep_embeddings=True, include_embeddings=True)
    cs = chunks("d0", 6)
    run(s.add_chunks(cs))
    got = run(s.get_by_id("d0_chunk_2"))
    assert got.embedding == cs[2].embedding  # chroma_store.py:233-244: the stored fp32 values
    hit = run(s.search(query_embedding=cs[4].embedding, top_k=1))[0][0]
    assert hit.id == "d0_chunk_4" and hit.embedding == cs[4].embedding
    s.flush()
    s2 = make_store(tmp_path, dtype="bf16", keep_embeddings=True)
    assert run(s2.get_by_id("d0_chunk_5")).embedding == cs[5].embedding


def test_concurrent_retrieves_coalesce_into_one_launch(tmp_path):
    """64 concurrent VectorRetriever.retrieve calls (the reference's one-query-per-call pattern,
    base_retriever.py:58-63) give the results of 64 sequential calls with one index search."""
    s = make_store(tmp_path)
    run(s.add_chunks(chunks("d0", 500, dim=16)))
    rng = np.random.default_rng(4)
    table = {f"q{i}": rng.standard_normal(16).astype(np.float32) for i in range(64)}

    class Emb:
        async def embed_query(self, q):
            return table[q].tolist()

    ret = VectorRetriever(s, Emb(), RetrieverConfig(top_k=5, similarity_threshold=0.0))
    seq = [run(ret.retrieve(q, top_k=3 + i % 5)) for i, q in enumerate(table)]
    before, launches = s._index.searches, s._batcher.launches

    async def concurrent():
        return await asyncio.gather(*[ret.retrieve(q, top_k=3 + i % 5) for i, q in enumerate(table)])

    par = run(concurrent())
    assert s._index.searches - before == 1 and s._batcher.launches - launches == 1
    assert [[(r.chunk.id, r.score, r.rank) for r in x] for x in par] == [[(r.chunk.id, r.score, r.rank) for r in x]
                                                                         for x in seq]

    # different filters go to different launches; results still per-call exact
    async def mixed():
        return await asyncio.gather(*[s.search(query_embedding=table[q].tolist(), top_k=4,
                                               filters={"chunk_index": {"$lt": 250}} if i % 2 else None)
                                      for i, q in enumerate(table)])

    before = s._index.searches
    res = run(mixed())
    assert s._index.searches - before == 2
    for i, r in enumerate(res):
        if i % 2:
            assert all(c.chunk_index < 250 for c, _ in r)


def test_filter_cache_extends_over_appended_rows():
    cols = F.MetadataColumns()
    rng = np.random.default_rng(1)
    metas = []

    def brute(w):
        def ok(m):
            return all((m.get(k) == v and not isinstance(m.get(k), bool)) if not isinstance(v, dict)
                       else (k in m and m[k] > v["$gt"]) for k, v in w.items())
        return np.array([ok(m) for m in metas], bool)

    wheres = [{"src": "a"}, {"src": "b", "n": {"$gt": 3}}, {"n": {"$gt": 5}}]
    for step in range(5):
        new = [{"src": ["a", "b", "c"][rng.integers(3)], "n": int(rng.integers(10))} if rng.random() < 0.9
               else {"other": 1} for _ in range(int(rng.integers(1, 200)))]
        metas.extend(new)
        cols.append(new)
        for w in wheres:  # cached after the first step, then extended
            np.testing.assert_array_equal(F.evaluate(w, cols), brute(w))
            words = F.evaluate_words(w, cols)
            assert len(words) == (len(metas) + 63) // 64


def test_journal_format_roundtrip(tmp_path):
    j = P.Journal(str(tmp_path / "x.journal"), fsync=False)
    v = np.arange(12, dtype=np.float32).reshape(3, 4)
    j.append_add([{"id": "a"}, None, {"id": "c"}], v)
    j.append_delete([5, 7])
    j.close()
    ops = list(P.Journal.replay(str(tmp_path / "x.journal")))
    assert ops[0][0] == "add" and ops[0][1] == [{"id": "a"}, None, {"id": "c"}]
    np.testing.assert_array_equal(ops[0][2], v)
    assert ops[1][0] == "del" and ops[1][1].tolist() == [5, 7]


# ---------------------------------------------------------------- concurrency fixes (round-2 advisor)
def test_rows_added_between_prep_and_run_of_filtered_search(tmp_path):
    """The filter bitmap is built when the search runs (under the store lock), not when it was queued:
    rows added in between cannot make it too short, and rows outside the filter are never returned."""
    s = make_store(tmp_path, persist=False)
    s.add_chunks_sync(chunks("a", 100))
    q = np.random.default_rng(3).standard_normal((4, 16)).astype(np.float32)
    prep = s._prep_search(q, 5, {"source": "src_a"})
    s.add_chunks_sync(chunks("b", 5000, seed=1))      # 100 -> 5100 rows: 2 -> 80 bitmap words
    res = s._assemble(prep, s._run_search(prep))
    assert all(len(r) == 5 and all(c.document_id == "a" for c, _ in r) for r in res)
    prep = s._prep_search(q, 5, {"source": "src_b"})
    res = s._assemble(prep, s._run_search(prep))
    assert all(len(r) == 5 and all(c.document_id == "b" for c, _ in r) for r in res)


def test_bad_query_dim_fails_alone(tmp_path):
    """A query of the wrong length is refused before it is queued; the other concurrent searches of the
    same filter group complete (before: np.stack raised inside the drain task and every waiter hung)."""
    s = make_store(tmp_path, persist=False)
    s.add_chunks_sync(chunks("a", 50))
    good = np.random.default_rng(4).standard_normal((8, 16)).astype(np.float32)

    async def main():
        tasks = [asyncio.ensure_future(s.search(query_embedding=g.tolist(), top_k=3)) for g in good]
        bad = asyncio.ensure_future(s.search(query_embedding=[0.5] * 15, top_k=3))
        done = await asyncio.wait_for(asyncio.gather(*tasks, bad, return_exceptions=True), 30)
        return done

    out = run(main())
    assert isinstance(out[-1], ValueError)
    assert all(isinstance(r, list) and len(r) == 3 for r in out[:-1])


def test_clear_while_search_in_flight_drops_stale_rows(tmp_path):
    s = make_store(tmp_path, persist=False)
    s.add_chunks_sync(chunks("a", 50))
    q = np.random.default_rng(5).standard_normal((2, 16)).astype(np.float32)
    prep = s._prep_search(q, 5, None)
    ran = s._run_search(prep)
    s._clear_sync()
    s.add_chunks_sync(chunks("b", 3000, seed=2))      # new rows reuse the old row numbers
    assert s._assemble(prep, ran) == [[], []]


def test_mutators_do_not_block_the_event_loop(tmp_path):
    """add_chunks / delete / get_by_id wait for the store lock in a worker thread: while a search holds
    the lock (here: another thread), the event loop keeps running other tasks."""
    import threading

    s = make_store(tmp_path, persist=False)
    s.add_chunks_sync(chunks("a", 20))
    held, release = threading.Event(), threading.Event()

    def holder():
        with s._lock:
            held.set()
            release.wait(10)

    th = threading.Thread(target=holder)
    th.start()
    held.wait(10)

    async def main():
        ticks = 0
        add = asyncio.ensure_future(s.add_chunks(chunks("b", 3, seed=1)))
        get = asyncio.ensure_future(s.get_by_id("a_chunk_1"))
        for _ in range(20):
            await asyncio.sleep(0.005)
            ticks += 1
        assert not add.done() and not get.done()   # still waiting for the lock ...
        release.set()                               # ... while the loop ran 20 ticks
        await add
        assert (await get).id == "a_chunk_1"
        return ticks

    assert run(main()) == 20
    th.join()
    assert run(s.count()) == 23


def test_sibling_collection_files_survive_clear(tmp_path):
    def store(name):
        cfg = VectorStoreConfig(backend="hip", collection_name=name, persist_directory=str(tmp_path),
                                index_params={"dtype": "f32", "persist": True, "fsync": False})
        return HipVectorStore(cfg, index_factory=lambda dim: OracleIndex(dim, "f32"),
                              index_loader=lambda path, dim, dt, metric: OracleIndex.load(path))

    a, b = store("docs"), store("docs.gov")
    run(a.add_chunks(chunks("x", 10)))
    run(b.add_chunks(chunks("y", 10, seed=1)))
    before = set(os.listdir(tmp_path))
    run(a.clear())
    left = set(os.listdir(tmp_path))
    assert {f for f in before if f.startswith("docs.gov.")} <= left
    assert not any(f.startswith("docs.") and not f.startswith("docs.gov.") for f in left)
    assert run(store("docs.gov").count()) == 10



# ---------------------------------------------------------------- native asynchronous launches (eventfd)
def make_async_store(tmp_path, **params):
    cfg = VectorStoreConfig(backend="hip", collection_name="kb", persist_directory=str(tmp_path),
                            index_params={"dtype": "f32", "persist": False, "fsync": False, **params})
    holder = {}

    def factory(dim):
        holder["idx"] = AsyncOracleIndex(dim, "f32")
        return holder["idx"]

    return HipVectorStore(cfg, index_factory=factory), holder


def test_native_async_launches_match_sequential(tmp_path):
    """Unfiltered concurrent searches go through the asynchronous entry point (launched from the event
    loop, completion by eventfd) and give exactly the sequential answers; filtered ones take the worker
    path in the same drain."""
    s, holder = make_async_store(tmp_path, max_batch=16)
    s.add_chunks_sync(chunks("a", 300) + chunks("b", 200, seed=1))
    q = np.random.default_rng(11).standard_normal((80, 16)).astype(np.float32)
    want = [[(c.id, sc) for c, sc in r] for r in s.search_batch(q, 7)]
    want_f = [[(c.id, sc) for c, sc in r] for r in s.search_batch(q[:8], 5, {"source": "src_b"})]

    async def main():
        un = [s.search(query_embedding=x.tolist(), top_k=7) for x in q]
        fi = [s.search(query_embedding=x.tolist(), top_k=5, filters={"source": "src_b"}) for x in q[:8]]
        return await asyncio.gather(*un, *fi)

    out = run(main())
    assert [[(c.id, sc) for c, sc in r] for r in out[:80]] == want
    assert [[(c.id, sc) for c, sc in r] for r in out[80:]] == want_f
    assert s._batcher.native_launches >= 5  # 80 queries / max_batch 16
    assert not holder["idx"].tickets       # every native batch collected
    s.close()


def test_native_async_busy_handle_and_clear(tmp_path):
    """A busy handle sends the batch to the worker path; a clear while native batches are in flight
    resolves them with no rows (their rows are gone) instead of resolving through the new tables."""
    s, holder = make_async_store(tmp_path, max_batch=8)
    s.add_chunks_sync(chunks("a", 100))
    q = np.random.default_rng(12).standard_normal((16, 16)).astype(np.float32)
    holder["idx"].busy = True

    async def searches():
        return await asyncio.gather(*[s.search(query_embedding=x.tolist(), top_k=3) for x in q])

    out = run(searches())
    assert all(len(r) == 3 for r in out) and s._batcher.native_launches == 0
    holder["idx"].busy = False
    holder["idx"].delay = 0.05

    async def clear_mid_flight():
        tasks = [asyncio.ensure_future(s.search(query_embedding=x.tolist(), top_k=3)) for x in q]
        await asyncio.sleep(0.01)          # both native batches are in flight
        await s.clear()
        await s.add_chunks(chunks("z", 50, seed=3))
        return await asyncio.gather(*tasks)

    out = run(clear_mid_flight())
    assert s._batcher.native_launches == 2
    assert all(r == [] for r in out)
    s.close()


def test_native_async_fallback_collected_off_loop(tmp_path):
    """A batch whose collect would run the exact fallback (poll state 2: a synchronous corpus pass) is collected
    in a worker thread, never on the event loop; every answer equals the sequential search."""
    import threading
    import time

    s, holder = make_async_store(tmp_path, max_batch=8)
    s.add_chunks_sync(chunks("a", 300))
    idx = holder["idx"]
    q = np.random.default_rng(13).standard_normal((32, 16)).astype(np.float32)
    want = [[(c.id, sc) for c, sc in r] for r in s.search_batch(q, 4)]
    where = {}
    submit0, collect0 = idx.search_submit_host, idx.search_collect

    def submit(qq, k, fd=-1):
        t = submit0(qq, k, fd)
        if t == 1:
            idx.needs_fallback.add(t)
        return t

    def collect(t, B, k):
        where[t] = threading.get_ident()
        if t in idx.needs_fallback:
            time.sleep(0.05)  # the fallback's corpus pass
        return collect0(t, B, k)

    idx.search_submit_host, idx.search_collect = submit, collect

    async def main():
        where["loop"] = threading.get_ident()
        return await asyncio.gather(*[s.search(query_embedding=x.tolist(), top_k=4) for x in q])

    out = run(main())
    assert [[(c.id, sc) for c, sc in r] for r in out] == want
    # 4 batches; a submit that finds the store lock held by the fallback's worker-thread collect takes the worker
    # path itself (never waits on the loop) -- how many do depends on the timing (a loaded host: all three), so
    # only batch 1 is certain to be native
    assert s._batcher.launches == 4 and s._batcher.native_launches >= 1 and not idx.tickets
    assert where[1] != where["loop"]                                   # the fallback batch: never on the loop
    s.close()


def test_native_async_collect_out_of_order_then_submit(tmp_path):
    """The ADVICE r03 sequence: A and B in flight, B collected first (A's collect moved to a worker: a mutation
    held the store), then a third batch is submitted while A is still outstanding -- it must take the free slot,
    not fail; A is then collected (blocking) with its own answer."""
    s, holder = make_async_store(tmp_path, max_batch=8)
    s.add_chunks_sync(chunks("a", 200))
    q = np.random.default_rng(14).standard_normal((3, 4, 16)).astype(np.float32)
    want = [[[(c.id, sc) for c, sc in r] for r in s.search_batch(q[i], 5)] for i in range(3)]

    async def main():
        loop = asyncio.get_running_loop()
        b = s._batcher
        ia = s._submit_native(s._prep_search(q[0], 5, None), b, loop)
        ib = s._submit_native(s._prep_search(q[1], 5, None), b, loop)
        import threading

        held, release = threading.Event(), threading.Event()

        def mutation():  # holds the store lock from another thread (the store's lock is re-entrant)
            with s._lock:
                held.set()
                release.wait(5)

        th = threading.Thread(target=mutation)
        th.start()
        held.wait(5)
        assert s._collect_native(ia, blocking=False) is None  # A's non-blocking collect declines
        release.set()
        th.join()
        rb = s._collect_native(ib, blocking=False)
        ic = s._submit_native(s._prep_search(q[2], 5, None), b, loop)
        assert ic is not None  # the freed slot, while A is outstanding
        ra = await asyncio.to_thread(s._collect_native, ia, True)
        rc = s._collect_native(ic, blocking=True)
        return [s._assemble(s._prep_search(q[i], 5, None), r) for i, r in enumerate((ra, rb, rc))]

    out = run(main())
    assert [[[(c.id, sc) for c, sc in r] for r in o] for o in out] == want
    s.close()


def test_store_leaves_the_collector_alone(tmp_path, monkeypatch):
    """The library sets no process-wide collector policy: no gc.freeze after bulk loads, no
    gc.disable; a serving application that wants its startup heap frozen calls gc.freeze() itself."""
    import gc

    calls = []
    for name in ("freeze", "disable"):
        monkeypatch.setattr(gc, name, lambda name=name: calls.append(name))
    s = make_store(tmp_path)
    s.add_chunks_sync(chunks("a", 300))
    with s.deferred_save():
        s.add_chunks_sync(chunks("b", 300, seed=1))
    assert not calls and gc.isenabled()


def test_cancelled_search_leaves_its_batch_alone(tmp_path):
    """One client cancelling its search (a request timeout) cancels only its own future: the other queries of
    the same native batch get their answers, the batch is still collected, and the store keeps serving."""
    s, holder = make_async_store(tmp_path, max_batch=16)
    s.add_chunks_sync(chunks("a", 200))
    q = np.random.default_rng(13).standard_normal((12, 16)).astype(np.float32)
    want = [[(c.id, sc) for c, sc in r] for r in s.search_batch(q, 4)]
    holder["idx"].delay = 0.05

    async def main():
        tasks = [asyncio.ensure_future(s.search(query_embedding=x.tolist(), top_k=4)) for x in q]
        await asyncio.sleep(0.01)  # the batch is in flight
        tasks[3].cancel()
        done = await asyncio.gather(*tasks, return_exceptions=True)
        again = await s.search(query_embedding=q[0].tolist(), top_k=4)
        return done, again

    done, again = run(main())
    assert isinstance(done[3], asyncio.CancelledError)
    assert [[(c.id, sc) for c, sc in r] for i, r in enumerate(done) if i != 3] == \
        [w for i, w in enumerate(want) if i != 3]
    assert [(c.id, sc) for c, sc in again] == want[0]
    assert s._batcher.native_launches >= 1 and not holder["idx"].tickets
    s.close()


@pytest.mark.parametrize("launched", [False, True])
def test_a_closed_event_loop_does_not_strand_the_store(tmp_path, launched):
    """asyncio.run ending with a search queued (or a native launch in flight) used to leave the batcher 'running'
    for a loop that no longer exists, so every later search, on any loop, waited forever.  The next loop finishes
    the dead loop's launches (blocking collects, their eventfd counts dropped) and serves normally."""
    s, holder = make_async_store(tmp_path, max_batch=8)
    s.add_chunks_sync(chunks("a", 60))
    q = np.random.default_rng(14).standard_normal((2, 16)).astype(np.float32)
    want = [[(c.id, sc) for c, sc in r] for r in s.search_batch(q, 3)]
    holder["idx"].delay = 0.05 if launched else 0.0

    async def leave():
        s._batcher.submit(q[0], 3, None)  # queued, never awaited
        if launched:
            await asyncio.sleep(0.01)  # the drain has launched it natively; the loop then closes under it

    run(leave())
    # queued only: the dead loop's drain never ran ('running' for good); launched: the drain was cancelled with
    # the native launch outstanding (its completion would resolve a future of the closed loop)
    assert s._batcher.running if not launched else len(s._batcher._native) == 1

    async def again():
        return await asyncio.wait_for(asyncio.gather(*[s.search(query_embedding=x.tolist(), top_k=3) for x in q]), 10)

    got = run(again())
    assert [[(c.id, sc) for c, sc in r] for r in got] == want
    assert not holder["idx"].tickets and not s._batcher._native and not s._batcher.running
    s.close()

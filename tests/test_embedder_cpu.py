"""CPU: host logic of the in-process embedder and the GPU ingest slice.

* HashWordTokenizer: HF-style padding / truncation / special tokens.
* TorchRocmEmbedder: prefixes, instruction-token count, batching -- with the K7 kernel
  replaced by the torch restatement (tests/embed_ref.py) so the rest runs on CPU; the
  K7 kernel itself is checked against the same restatement in test_gpu_embedder.py.
* GpuIngestor: chunk ids / metadata as processors.py:387-407, delete-before-add,
  batches spanning documents (oracle-backed index, host-list embedder).
"""
import asyncio
import os

import numpy as np
import pytest
import torch

from embed_ref import ref_mean_pooling, ref_passages, ref_queries
from fake_index import OracleIndex
from hiprag.rag import ChunkingConfig, Document, HipVectorStore, VectorStoreConfig
from hiprag.rag.ingest import GpuIngestor, make_chunks
from hiprag.rag.rocm_embedder import HashWordTokenizer, TorchRocmEmbedder


def run(c):
    return asyncio.run(c)


def test_hash_tokenizer_hf_semantics():
    tok = HashWordTokenizer()
    one = tok("Hello, world!", add_special_tokens=True)["input_ids"]
    assert one[0] == 101 and one[-1] == 102 and len(one) == 6
    assert tok("", add_special_tokens=True)["input_ids"] == [101, 102]
    assert tok("", add_special_tokens=False)["input_ids"] == []
    assert tok("hello")["input_ids"][1] == tok("HELLO")["input_ids"][1]
    b = tok(["a b c d e f", "x"], padding=True, truncation=True, max_length=5, return_tensors="pt")
    assert b["input_ids"].shape == (2, 5) and b["attention_mask"].tolist() == [[1] * 5, [1, 1, 1, 0, 0]]
    assert b["input_ids"][0, -1] == 102 and b["input_ids"][1, -1] == 0


def test_hash_tokenizer_cached_ids_match_plain_crc32():
    """The word-id cache and the numpy padding give exactly the ids of the plain definition
    (crc32 of each lower-cased \\w+ / punctuation token), non-ASCII and truncation included."""
    import re
    import zlib

    word = re.compile(r"\w+|[^\w\s]", re.UNICODE)
    rng = np.random.default_rng(3)
    alpha = list("abcXYZ019_äÖß€ ,.!?\t\n")
    texts = ["".join(rng.choice(alpha, size=int(rng.integers(0, 300)))) for _ in range(40)] + ["", "   "]
    tok = HashWordTokenizer()
    tok._cache_max = 50  # exercise the cache reset too
    for max_length in (8, 512):
        got = tok(texts, padding=True, truncation=True, max_length=max_length, return_tensors="pt")
        want = [[101, *[1000 + zlib.crc32(w.encode()) % 29522 for w in word.findall(t.lower())][:max_length - 2], 102]
                for t in texts]
        width = max(map(len, want))
        assert got["input_ids"].tolist() == [s + [0] * (width - len(s)) for s in want]
        assert got["attention_mask"].tolist() == [[1] * len(s) + [0] * (width - len(s)) for s in want]
        assert got["input_ids"].dtype == torch.long and got["attention_mask"].dtype == torch.long


class CpuEmbedder(TorchRocmEmbedder):
    def _pool(self, hidden, mask, n_instr):
        m = mask.clone()
        m[:, :n_instr] = 0
        return torch.nn.functional.normalize(ref_mean_pooling(hidden, m), dim=-1)


@pytest.fixture(scope="module")
def cpu_emb():
    return CpuEmbedder(preset="tiny", device="cpu", batch_size=3, max_length=64)


def test_embedder_matches_reference_encode_on_cpu(cpu_emb):
    texts = ["the quick brown fox", "jumps over", "the lazy dog " * 10, "a", "retrieval augmented generation"]
    got = cpu_emb.encode_passages(texts)
    ref = torch.cat([ref_passages(cpu_emb, texts[i:i + 3]) for i in range(0, 5, 3)])
    torch.testing.assert_close(got, ref, rtol=0, atol=1e-6)
    q = cpu_emb.encode_queries(["what is a fox?", "dog"])
    torch.testing.assert_close(q, ref_queries(cpu_emb, ["what is a fox?", "dog"]), rtol=0, atol=1e-6)
    assert cpu_emb.query_instruction.startswith("Instruction: Given a search query") and \
        cpu_emb.query_instruction.endswith(" \nQuery:")
    # the empty passage instruction still masks the tokenizer's special tokens (mdx:98-107 quirk)
    assert cpu_emb._n_instruction_tokens("") == 2
    v = run(cpu_emb.embed_query("dog"))
    assert isinstance(v, list) and len(v) == 256 and abs(np.linalg.norm(v) - 1) < 1e-5
    assert len(run(cpu_emb.embed_texts(texts))) == 5
    assert cpu_emb.max_length == 64


def test_concurrent_embed_query_calls_share_forwards(cpu_emb):
    """The reference's retrieve() embeds one query per call; concurrent calls are coalesced into forwards of up to
    batch_size queries (run in the embedder's worker thread), each caller getting its own query's vector; a
    cancelled call leaves the rest of its forward alone."""
    qs = [f"query number {i} about w{i * 7 % 13}" for i in range(8)]
    want = cpu_emb.encode_queries(qs).numpy()
    co = cpu_emb._coalescer
    f0, n0 = co.forwards, co.queries

    async def main():
        tasks = [asyncio.ensure_future(cpu_emb.embed_query(q)) for q in qs]
        await asyncio.sleep(0)  # every call has queued its query
        tasks[5].cancel()
        return await asyncio.gather(*tasks, return_exceptions=True)

    got = run(main())
    assert isinstance(got[5], asyncio.CancelledError)
    for i, v in enumerate(got):
        if i != 5:
            assert isinstance(v, list) and len(v) == want.shape[1]
            np.testing.assert_allclose(v, want[i], rtol=0, atol=1e-5)
    # 8 calls, batch_size 3: at most ceil(7 / 3) + 1 forwards, never one per call
    assert co.queries - n0 in (7, 8) and co.forwards - f0 <= 4
    # a failing forward reaches every caller of its batch, and the coalescer keeps serving
    inner = cpu_emb._query_lists
    cpu_emb._query_lists = lambda q: (_ for _ in ()).throw(RuntimeError("forward failed"))
    try:
        async def two():
            return await asyncio.gather(*[cpu_emb.embed_query(q) for q in qs[:2]], return_exceptions=True)

        bad = run(two())
    finally:
        cpu_emb._query_lists = inner
    assert all(isinstance(e, RuntimeError) for e in bad)
    np.testing.assert_allclose(run(cpu_emb.embed_query(qs[0])), want[0], rtol=0, atol=1e-5)


def test_coalescer_survives_a_loop_that_stopped_before_its_drain(cpu_emb):
    """A loop that ends right after queueing a query (its drain never ran) does not strand the next loop's calls."""
    co = cpu_emb._coalescer

    async def queue_and_leave():
        co.submit("left behind")  # queued (never awaited); the loop closes before its drain finishes

    run(queue_and_leave())
    v = run(asyncio.wait_for(cpu_emb.embed_query("dog"), 30))
    np.testing.assert_allclose(v, cpu_emb.encode_queries(["dog"])[0].numpy(), rtol=0, atol=1e-5)
    live = [lq for loop, lq in list(co._queues.items()) if not loop.is_closed()]
    assert all(not lq.running and not lq.pending for lq in live)


def test_coalescer_serves_two_running_loops_apart(cpu_emb):
    """two event loops running at once in two threads each get their own queue and drain -- every
    future is resolved on its own loop, and neither drain takes the other loop's queries."""
    import threading

    qs = [f"thread query {i} w{i % 5}" for i in range(12)]
    want = cpu_emb.encode_queries(qs).numpy()
    out, errs = {}, []
    gate = threading.Barrier(2)

    def worker(t):
        async def main():
            gate.wait(10)  # both loops are running before either queues
            mine = qs[t::2]
            got = await asyncio.gather(*[cpu_emb.embed_query(q) for q in mine])
            assert not cpu_emb._coalescer.pending  # (this loop's queue)
            return mine, got

        try:
            out[t] = asyncio.run(asyncio.wait_for(main(), 60))
        except BaseException as e:  # noqa: BLE001
            errs.append(e)

    th = [threading.Thread(target=worker, args=(t,)) for t in range(2)]
    for x in th:
        x.start()
    for x in th:
        x.join(120)
    assert not errs, errs
    for t in range(2):
        mine, got = out[t]
        for q, v in zip(mine, got):
            np.testing.assert_allclose(v, want[qs.index(q)], rtol=0, atol=1e-5)


def test_default_embedder_leaves_tunableop_alone(cpu_emb, monkeypatch):
    """constructing an embedder does not touch the process's TunableOp state (tuned GEMMs are
    opt-in), and even when asked, an application's own TunableOp setup (enabled already, or PYTORCH_TUNABLEOP_*
    set) is left as it is; when it does act it never disables TunableOp, never renames its results file and writes
    nothing on exit.  torch.cuda.tunable needs a GPU, so a recorder stands in for it here."""
    import sys
    import types

    import torch

    from hiprag.rag import rocm_embedder as E

    calls = []
    state = {"enabled": False}
    fake = types.SimpleNamespace(
        is_enabled=lambda: state["enabled"],
        enable=lambda on=True: calls.append(("enable", on)),
        tuning_enable=lambda on=True: calls.append(("tuning_enable", on)),
        write_file_on_exit=lambda on: calls.append(("write_file_on_exit", on)),
        set_filename=lambda *a: calls.append(("set_filename",) + a),
        read_file=lambda path=None: calls.append(("read_file",)) or True)
    monkeypatch.setitem(sys.modules, "torch.cuda.tunable", fake)
    monkeypatch.setattr(torch.cuda, "tunable", fake, raising=False)
    monkeypatch.setattr(torch.cuda, "is_available", lambda: True)
    for k in [k for k in os.environ if k.startswith("PYTORCH_TUNABLEOP_")]:
        monkeypatch.delenv(k)
    monkeypatch.delenv("HIPRAG_TUNED_GEMMS", raising=False)

    # a default embedder never calls it
    monkeypatch.setattr(E, "enable_tuned_gemms", lambda *a, **k: (_ for _ in ()).throw(AssertionError("called")))
    emb = TorchRocmEmbedder(model=cpu_emb.model, tokenizer=cpu_emb.tokenizer, device="cpu", max_length=64)
    assert emb.tuned_gemms is False
    monkeypatch.undo()
    monkeypatch.setitem(sys.modules, "torch.cuda.tunable", fake)
    monkeypatch.setattr(torch.cuda, "tunable", fake, raising=False)
    monkeypatch.setattr(torch.cuda, "is_available", lambda: True)
    for k in [k for k in os.environ if k.startswith("PYTORCH_TUNABLEOP_")]:
        monkeypatch.delenv(k)

    state["enabled"] = True  # the application enabled TunableOp itself
    assert E.enable_tuned_gemms() is False and calls == []
    state["enabled"] = False
    monkeypatch.setenv("PYTORCH_TUNABLEOP_FILENAME", "/tmp/app_results.csv")  # ... or configured it
    assert E.enable_tuned_gemms() is False and calls == []
    monkeypatch.delenv("PYTORCH_TUNABLEOP_FILENAME")
    assert E.enable_tuned_gemms() is True  # nothing configured: read the shipped results, tuning off, no exit write
    assert calls == [("tuning_enable", False), ("write_file_on_exit", False), ("read_file",), ("enable", True)]
    calls.clear()
    del fake.write_file_on_exit  # (torch 2.10 has no write_file_on_exit: tuning off is what keeps the file unwritten)
    assert E.enable_tuned_gemms() is True
    assert calls == [("tuning_enable", False), ("read_file",), ("enable", True)]


def test_fused_retrieve_matches_two_step_path(cpu_emb, tmp_path):
    """VectorRetriever over hiprag's embedder and store fuses concurrent retrieve() calls into cohorts (one forward
    whose output goes straight into one store search, retriever._FusedRetrieve): same chunks, ranks and scores as
    the reference's two awaits (embed_query, then store.search) for the same queries, per-call top_k and
    thresholds respected, filtered calls and a reranker keep the two-step path."""
    from hiprag.rag import RetrieverConfig, VectorRetriever
    from hiprag.rag.base import Chunk

    store = HipVectorStore(VectorStoreConfig(backend="hip", collection_name="fused", persist_directory=str(tmp_path),
                                             index_params={"dtype": "f32", "persist": False}),
                           index_factory=lambda d: OracleIndex(d, "f32"))
    docs = [f"document {i} about w{i % 13} and w{(i * 7) % 31} with details {i * 3}" for i in range(120)]
    vecs = cpu_emb.encode_passages(docs).numpy()
    store.add_chunks_sync([Chunk(id=f"c{i}", document_id=f"d{i // 10}", content=docs[i], chunk_index=i % 10,
                                 metadata={"grp": f"g{i % 2}"}, embedding=vecs[i].tolist()) for i in range(120)])
    cfg = RetrieverConfig(top_k=5, similarity_threshold=0.0)
    ret = VectorRetriever(store, cpu_emb, cfg)
    two = VectorRetriever(store, cpu_emb, cfg)
    two._fused = None
    assert ret._fused is not None
    qs = [(f"what about w{i % 13} and details {i}", 3 + i % 5) for i in range(11)]

    async def fused():
        return await asyncio.gather(*[ret.retrieve(q, top_k=k) for q, k in qs],
                                    ret.retrieve(qs[0][0], top_k=4, filters={"grp": "g1"}))

    got = run(fused())
    assert ret._fused.queries == len(qs) and ret._fused.cohorts < len(qs)  # the filtered call took the two-step path
    for (q, k), res in zip(qs, got):
        want = run(two.retrieve(q, top_k=k))
        assert [r.chunk.id for r in res] == [r.chunk.id for r in want] and [r.rank for r in res] == list(range(1, k + 1))
        np.testing.assert_allclose([r.score for r in res], [r.score for r in want], rtol=0, atol=1e-5)
    want_f = run(two.retrieve(qs[0][0], top_k=4, filters={"grp": "g1"}))
    assert [r.chunk.id for r in got[-1]] == [r.chunk.id for r in want_f]
    assert all(r.chunk.metadata["grp"] == "g1" for r in got[-1])
    high = run(ret.retrieve(qs[1][0], top_k=5, similarity_threshold=0.99))  # threshold filtering after the ranks
    assert all(r.score >= 0.99 for r in high)
    # one cohort, different thresholds and top_k per call: each call's hits are the two-step path's, ranks counted
    # before its own threshold drops any (base_retriever.py:66-72)
    mixed = [(qs[2][0], 6, 0.0), (qs[2][0], 6, 0.5), (qs[3][0], 2, 0.3), (qs[4][0], 7, -1.0)]

    async def fused_mixed():  # (concurrent calls on one loop: formed into one cohort by the next loop iteration)
        return await asyncio.gather(*[ret.retrieve(q, top_k=k, similarity_threshold=t) for q, k, t in mixed])

    got_m = run(fused_mixed())
    for (q, k, t), res in zip(mixed, got_m):
        want = run(two.retrieve(q, top_k=k, similarity_threshold=t))
        assert [(r.chunk.id, r.rank) for r in res] == [(r.chunk.id, r.rank) for r in want]
    assert len(got_m[1]) <= len(got_m[0]) and [r.rank for r in got_m[0]] == list(range(1, 7))
    ret._fused.close()

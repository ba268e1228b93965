"""CPU: host logic of the in-process embedder and the GPU ingest slice.

* HashWordTokenizer: HF-style padding / truncation / special tokens.
* TorchRocmEmbedder: prefixes, instruction-token count, batching -- with the K7 kernel
  replaced by the torch restatement (tests/embed_ref.py) so the rest runs on CPU; the
  K7 kernel itself is checked against the same restatement in test_gpu_embedder.py.
* GpuIngestor: chunk ids / metadata as processors.py:387-407, delete-before-add,
  batches spanning documents (oracle-backed index, host-list embedder).
"""
import asyncio

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
    assert not co.running and not co.pending


def test_embedder_rejects_missing_local_model():
    with pytest.raises(FileNotFoundError):
        TorchRocmEmbedder("/nonexistent/model", device="cpu")


def test_make_chunks_matches_processor_convention():
    doc = Document(id="report.pdf", content="", metadata={"source": "s3", "_private": 1})
    ch = make_chunks(doc, ["a", "b"], {"kb": 7})
    assert [c.id for c in ch] == ["report.pdf_chunk_0", "report.pdf_chunk_1"]
    assert ch[1].metadata == {"source": "s3", "index_type": "index_content", "kb": 7} and ch[1].chunk_index == 1
    doc2 = Document(id="d", content="", metadata={"index_type": "index_summary"})
    assert make_chunks(doc2, ["x"])[0].metadata["index_type"] == "index_summary"


class HashEmbedder:
    """Host-list embedder: deterministic vectors per text."""
    batch_size = 4

    def __init__(self):
        self.batches = []

    async def embed_texts(self, texts):
        self.batches.append(len(texts))
        return [np.random.default_rng(abs(hash(t)) % 2**32).standard_normal(16).tolist() for t in texts]


def test_ingestor_batches_across_documents_and_replaces_old_chunks(tmp_path):
    cfg = VectorStoreConfig(backend="hip", collection_name="kb", persist_directory=str(tmp_path),
                            index_params={"dtype": "f32", "persist": False})
    store = HipVectorStore(cfg, index_factory=lambda d: OracleIndex(d, "f32"))
    emb = HashEmbedder()
    ing = GpuIngestor(store, emb, chunking=ChunkingConfig(chunk_size=100, chunk_overlap=0))
    docs = [Document(id=f"doc{i}", content=" ".join(f"word{j}" for j in range(30 * i + 2)), metadata={"n": i})
            for i in range(6)]
    n = run(ing.ingest(docs))
    # every document's chunks + its summary vector (processors.py:559-561, :423-464)
    assert n + 6 == run(store.count()) and sum(emb.batches) == n + 6 and max(emb.batches) == 4
    assert all(b == 4 for b in emb.batches[:-1])
    c = run(store.get_by_id("doc3_chunk_0"))
    assert c.metadata["n"] == 3 and c.metadata["index_type"] == "index_content"
    sm = run(store.get_by_id("doc3_summary"))
    assert sm.content == "doc3\n" and sm.chunk_index == -1
    assert sm.metadata == {"document_id": "doc3", "chunk_index": -1, "n": 3, "index_type": "index_summary"}
    # re-ingesting a document replaces its chunks and its summary
    before = run(store.count())
    old = len(store._doc_rows["doc5"])
    m = run(ing.chunk_and_store(Document(id="doc5", content="short text", metadata={"source": "s.pdf",
                                                                                       "summary": "about x"})))
    assert run(store.count()) == before - old + m + 1 and len(store._doc_rows["doc5"]) == m + 1
    assert run(store.get_by_id("doc5_summary")).content == "s.pdf\nabout x"
    no_sum = GpuIngestor(store, emb, summary_index=False)
    assert run(no_sum.chunk_and_store(Document(id="doc9", content="a b c", metadata={}))) == 1
    assert run(store.get_by_id("doc9_summary")) is None
    # chunklevel.md documents take the hierarchical splitter (processors.py:371-379); "_" keys stay out
    hc = ing.split(Document(id="h", content="# T\n## S\nline a\nline b", metadata={"_use_hierarchical_splitter": True,
                                                                                   "source": "c.md"}))
    assert [c.content for c in hc] == ["# T\n## S\n\nline a\nline b"]
    assert hc[0].metadata == {"source": "c.md", "index_type": "index_content"} and hc[0].id == "h_chunk_0"


def test_hash_tokenizer_native_text_kernel_matches_python():
    """hr_hash_words (the host text kernel ASCII batches take) gives the ids of the re + zlib path:
    every ASCII whitespace class, punctuation, digits, underscores, control bytes, truncation with
    and without special tokens; batches with a non-ASCII text stay on the Python path."""
    import random

    from hiprag.rag import rocm_embedder as re_mod

    rnd = random.Random(11)
    alpha = "abcXYZ0189_ ,.!?;:'\"()-\t\n\x0b\x0c\r\x1c\x1d\x1e\x1f\x7f\x00@#$%^&*[]{}|\\/~`"
    texts = ["".join(rnd.choice(alpha) for _ in range(rnd.randint(0, 400))) for _ in range(60)] + ["", " \t "]
    tok = HashWordTokenizer()
    old = re_mod._NATIVE_TOK
    try:
        for max_length, special in ((8, True), (512, True), (None, True), (6, False)):
            kw = dict(padding=True, truncation=max_length is not None, max_length=max_length, return_tensors="pt",
                      add_special_tokens=special)
            re_mod._NATIVE_TOK = True
            assert tok._native_batch(texts, None, special) is not None
            a = tok(texts, **kw)
            re_mod._NATIVE_TOK = False
            b = tok(texts, **kw)
            assert torch.equal(a["input_ids"], b["input_ids"]) and torch.equal(a["attention_mask"], b["attention_mask"])
        assert tok._native_batch(texts + ["naïve"], None, True) is None
    finally:
        re_mod._NATIVE_TOK = old


def test_ingest_keeps_the_cyclic_gc_enabled(tmp_path):
    """The ingest no longer switches the collector off for its duration (a global side effect
    on every other coroutine of the serving process)."""
    import gc

    seen = []

    class GcProbe(HashEmbedder):
        async def embed_texts(self, texts):
            seen.append(gc.isenabled())
            return await super().embed_texts(texts)

    cfg = VectorStoreConfig(backend="hip", collection_name="kb", persist_directory=str(tmp_path),
                            index_params={"dtype": "f32", "persist": False})
    store = HipVectorStore(cfg, index_factory=lambda d: OracleIndex(d, "f32"))
    docs = [Document(id=f"d{i}", content="alpha beta gamma " * 20, metadata={}) for i in range(3)]
    run(GpuIngestor(store, GcProbe(), chunking=ChunkingConfig(chunk_size=100, chunk_overlap=0)).ingest(docs))
    assert seen and all(seen) and gc.isenabled()


def test_pack_pad_sequence_changes_no_real_row():
    """UnpaddedEncoder.pack(granule=64): one extra sequence of 1..64 pad tokens makes the token count a multiple of
    64 (the shapes graph replays are captured for); every sequence attends only to itself, so the real tokens'
    hidden states equal the unpadded pack's (fp32, CPU, SDPA per sequence), and `lengths` keeps the real ones."""
    import numpy as np
    import torch

    from hiprag.rag.encoder import UnpaddedEncoder
    from hiprag.rag.rocm_embedder import build_random_bert

    model = build_random_bert("tiny", seed=3).eval()
    enc = UnpaddedEncoder(model, use_varlen=False)
    rng = np.random.default_rng(0)
    lens = rng.integers(1, 20, 9)
    ids = np.zeros((9, 20), np.int64)
    mask = np.zeros((9, 20), np.int64)
    for i, n in enumerate(lens):
        ids[i, :n] = rng.integers(1, 30000, n)
        mask[i, :n] = 1
    with torch.inference_mode():
        p0 = enc.pack(ids, mask, device="cpu")
        p1 = enc.pack(ids, mask, device="cpu", granule=64)
        h0, h1 = enc.forward_packed(p0), enc.forward_packed(p1)
    n = int(lens.sum())
    assert int(p1.cu_host[-1]) % 64 == 0 and 1 <= int(p1.cu_host[-1]) - n <= 64
    np.testing.assert_array_equal(p1.lengths, lens)
    np.testing.assert_array_equal(p1.cu_host[:-1], p0.cu_host)
    torch.testing.assert_close(h1[:n], h0, rtol=1e-5, atol=1e-5)

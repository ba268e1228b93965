"""GPU: concurrency and resource-lifetime cases of the host layer.

* the query coalescer's first forward of a new shape is CAPTURED into a HIP graph on its worker thread
  while the event loop's thread launches the store's native searches -- with an empty graph cache, many concurrent
  VectorRetriever.retrieve calls (embed_query -> store.search, base_retriever.py:57-63) must return what the same
  vectors return searched one by one, and the vectors must be the embedder's.
* a CU-masked stream (hr_stream_create_cu_mask) used for the embedder and the search (the bench's
  CU split) and then destroyed (hr_stream_destroy) while tensors made on it are still alive: the process exits 0.
"""
import asyncio
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)


@pytest.mark.timeout(300)
def test_concurrent_retrieve_with_cold_graph_capture(tmp_path):
    from hiprag.rag import HipVectorStore, VectorStoreConfig
    from hiprag.rag.base import Chunk
    from hiprag.rag.rocm_embedder import TorchRocmEmbedder

    emb = TorchRocmEmbedder(preset="tiny", dtype="bfloat16", batch_size=32, max_length=128, seed=3)
    assert emb.graphed is not None and not emb.graphed.graphs  # cold: the first coalesced forward captures
    rng = np.random.default_rng(4)
    n, dim = 50_000, emb.dim
    rows = rng.standard_normal((n, dim)).astype(np.float32)
    cfg = VectorStoreConfig(backend="hip", collection_name="conc", persist_directory=str(tmp_path),
                            index_params={"dtype": "bf16", "persist": False, "max_batch": 16})
    store = HipVectorStore(cfg)
    store.add_chunks_sync([Chunk(id=f"c{i}", document_id=f"d{i // 50}", content=str(i), chunk_index=i % 50,
                                 metadata={}, embedding=rows[i].tolist()) for i in range(n)])
    texts = [f"question {i} about topic w{i % 17} and w{(i * 5) % 23}" for i in range(96)]

    async def retrieve(t):  # VectorRetriever.retrieve's two awaits (base_retriever.py:57-63), vector kept
        v = await emb.embed_query(t)
        return v, await store.search(query_embedding=v, top_k=10)

    async def many():
        return await asyncio.gather(*[retrieve(t) for t in texts])

    out = asyncio.run(many())
    assert emb.graphed.graphs and emb._coalescer.forwards < len(texts)  # coalesced forwards, graphs captured
    # the vectors are the embedder's (a batch of another size only changes GEMM rounding)
    ref = emb.encode_queries(texts).cpu().numpy()
    v = np.asarray([x for x, _ in out], np.float32)
    assert float((v * ref).sum(1).min()) > 0.999

    async def alone(x):
        return await store.search(query_embedding=x, top_k=10)

    for x, res in out:  # each concurrent answer == the same vector searched alone, on a quiet loop
        want = asyncio.run(alone(x))
        assert [c.id for c, _ in res] == [c.id for c, _ in want]
        assert [s for _, s in res] == [s for _, s in want]
    store.close()
    emb._coalescer.close()


@pytest.mark.timeout(200)
def test_cu_masked_streams_destroyed_then_clean_exit():
    proc = subprocess.run([sys.executable, "-u", os.path.join(REPO, "tools", "cu_stream_probe.py"), "split", "lib",
                           "alive"], timeout=150, capture_output=True, text=True)
    print(proc.stdout[-2000:], proc.stderr[-3000:])
    assert proc.returncode == 0, (proc.returncode, proc.stderr[-3000:])
    assert "destroyed" in proc.stdout and "exiting" in proc.stdout


@pytest.mark.timeout(300)
def test_fused_retrieve_on_gpu_matches_two_step(tmp_path):
    """The retriever's fused cohorts on the GPU (one bf16 forward whose (B, dim) output feeds hr_index_search_device
    directly) vs the reference's two awaits (embed_query lists -> store.search) over the same store: the same top-k
    wherever the two forwards' roundings do not reorder a near tie, scores within the bf16 forward's rounding."""
    from hiprag.rag import HipVectorStore, RetrieverConfig, VectorRetriever, VectorStoreConfig
    from hiprag.rag.base import Chunk
    from hiprag.rag.rocm_embedder import TorchRocmEmbedder

    emb = TorchRocmEmbedder(preset="tiny", dtype="bfloat16", batch_size=32, max_length=128, seed=5)
    docs = [f"passage {i} on subject w{i % 41} with w{(i * 11) % 97} and w{(i * 5) % 13}" for i in range(3000)]
    vecs = emb.encode_passages(docs).cpu().numpy()
    cfg = VectorStoreConfig(backend="hip", collection_name="fused", persist_directory=str(tmp_path),
                            index_params={"dtype": "f32", "persist": False, "max_batch": 32})
    store = HipVectorStore(cfg)
    store.add_chunks_sync([Chunk(id=f"c{i}", document_id=f"d{i // 30}", content=docs[i], chunk_index=i % 30,
                                 metadata={}, embedding=vecs[i].tolist()) for i in range(len(docs))])
    rc = RetrieverConfig(top_k=8, similarity_threshold=0.0)
    ret, two = VectorRetriever(store, emb, rc), VectorRetriever(store, emb, rc)
    two._fused = None
    assert ret._fused is not None
    qs = [f"what is said on subject w{i % 41} and w{(i * 3) % 97}" for i in range(100)]

    async def many(r):
        return await asyncio.gather(*[r.retrieve(q) for q in qs])

    got, want = asyncio.run(many(ret)), asyncio.run(many(two))
    assert ret._fused.cohorts >= 4 and ret._fused.queries == len(qs)
    same = sum([x.chunk.id for x in g] == [x.chunk.id for x in w] for g, w in zip(got, want))
    assert same >= 0.9 * len(qs), same
    for g, w in zip(got, want):
        assert len(g) == 8 and abs(g[0].score - w[0].score) < 2e-2
    store.close()
    ret._fused.close()

"""Profile target: the cross-encoder rerank of 8 queries x 100 passages (tools/bench_rerank.py stage 2)."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "youtu-rag_amd"), REPO]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from hiprag.rag import Chunk, RetrievalResult  # noqa: E402
from hiprag.rag.rerankers import TorchRocmReranker  # noqa: E402

bs = int(os.environ.get("RR_BATCH", 512))
rr = TorchRocmReranker(preset="bge-reranker-base", dtype="bfloat16", batch_size=bs, max_length=512)
vocab = [f"tok{i}" for i in range(20000)]
rng = np.random.default_rng(0)
work = []
for step in range(6):
    qs = [" ".join(rng.choice(vocab, 12)) for _ in range(8)]
    res = [[RetrievalResult(chunk=Chunk(id=f"{step}_{b}_{i}", document_id="d", content=" ".join(rng.choice(vocab, 110)),
                                        chunk_index=i), score=0.5, rank=i + 1) for i in range(100)] for b in range(8)]
    work.append((qs, res))
for qs, res in work[:2]:
    rr.rerank_batch(qs, res, top_k=10)
torch.cuda.synchronize()
t0 = time.perf_counter()
for qs, res in work[2:]:
    for r in res:  # warm passage token cache, so the timing below is the GPU part + pair assembly
        for x in r:
            rr._text_ids(x.chunk.content, cache=True)
t_tok = time.perf_counter() - t0
t0 = time.perf_counter()
for qs, res in work[2:]:
    rr.rerank_batch(qs, res, top_k=10)
torch.cuda.synchronize()
dt = (time.perf_counter() - t0) / 4
print(f"batch {bs}: {dt * 1e3:.1f} ms per 800 pairs ({800 / dt:.0f} pairs/s); tokenising 800 passages {t_tok / 4 * 1e3:.1f} ms",
      flush=True)

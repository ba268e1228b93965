"""In-process cross-encoder reranker behind BaseReranker (BASELINE config 5).

Replaces the reference's HTTP rerankers (OpenAIReranker, utu/rag/rerankers/openai_reranker.py
:67-214; ServiceReranker / TioneReranker, same contract) with the computation a reranking
server runs, in this process on the MI355X:

* every (query, passage) pair is tokenised as ``[CLS] query [SEP] passage [SEP]`` with
  ``longest_first`` truncation to ``max_length`` (the Hugging Face pair convention of
  cross-encoder rerankers); passage token ids are cached per content string, so a chunk that
  is reranked again is not re-tokenised;
* the cross-encoder forward (a sequence-classification transformer, one logit per pair) runs
  in PyTorch-ROCm over length-sorted batches of pairs from one or many queries (padding waste
  is bounded by the length spread of a batch, not of the whole request);
* relevance = sigmoid(logit) (the 0..1 ``relevance_score`` of the /rerank API);
* per query, the top ``top_n`` pairs by (relevance desc, original position asc) are selected by
  the HIP kernel ``hr_topk_records`` -- the order the reference takes from the service's
  response (openai_reranker.py:96-110) -- and returned as new ``RetrievalResult`` objects with
  ``rank`` = 1-based position.
Reference behaviour kept: empty input returns as is (:83-84); ``top_k`` None means all (:86);
any failure logs and returns ``results[:top_k]`` (:117-121).

No checkpoint can be downloaded here: ``model_name_or_path`` must be a local directory
(AutoModelForSequenceClassification with local_files_only); without one a seeded random-init
BERT classifier of the bge-reranker-base shape is built, with the offline HashWordTokenizer.
"""
from __future__ import annotations

import logging
import os

import numpy as np

from .. import _native
from .base import BaseReranker, RetrievalResult
from .rocm_embedder import PRESETS, HashWordTokenizer, fuse_encoder_layers

logger = logging.getLogger(__name__)

RERANK_PRESETS = {"bge-reranker-base": PRESETS["bge-base"], "bge-reranker-large": PRESETS["bge-large"],
                  "tiny": PRESETS["tiny"]}
_TORCH_DTYPES = {"float32": "float32", "fp32": "float32", "bfloat16": "bfloat16", "bf16": "bfloat16",
                 "float16": "float16", "fp16": "float16"}


def truncate_pair(a: list[int], b: list[int], max_length: int) -> tuple[list[int], list[int]]:
    """``longest_first`` truncation of a token-id pair to max_length including [CLS], [SEP], [SEP],
    as the Hugging Face tokenizers library does it: the shorter input is kept whole when the longer
    one can absorb the cut; otherwise both get half the budget, the longer (the second, on equal
    lengths) the odd token."""
    target = max(0, int(max_length) - 3)
    n1, n2 = len(a), len(b)
    if n1 + n2 <= target:
        return list(a), list(b)
    swap = n1 > n2
    if swap:
        n1, n2 = n2, n1
    n2 = n1 if n1 > target else max(n1, target - n1)
    if n1 + n2 > target:
        n1 = target // 2
        n2 = n1 + target % 2
    if swap:
        n1, n2 = n2, n1
    return list(a[:n1]), list(b[:n2])


def build_random_cross_encoder(preset: str = "bge-reranker-base", seed: int = 0, **overrides):
    """Seeded random-init BertForSequenceClassification (one logit per pair)."""
    import torch
    from transformers import BertConfig, BertForSequenceClassification

    cfg = dict(RERANK_PRESETS[preset])
    cfg.update(overrides)
    config = BertConfig(vocab_size=30522, max_position_embeddings=512, num_labels=1, **cfg)
    with torch.random.fork_rng(devices=[]):
        torch.manual_seed(seed)
        model = BertForSequenceClassification(config)
    return model


class TorchRocmReranker(BaseReranker):
    """BaseReranker running a cross-encoder in-process on an MI355X."""

    def __init__(self, model_name_or_path: str | None = None, *, model=None, tokenizer=None,
                 preset: str = "bge-reranker-base", batch_size: int = 256, max_length: int = 512, gpu_id: int = 0,
                 device=None, dtype: str = "bfloat16", seed: int = 0, cache_size: int = 1 << 20,
                 fused_layernorm: bool | None = None, **_ignored):
        import torch

        self.torch = torch
        if fused_layernorm is None:
            fused_layernorm = os.environ.get("HIPRAG_FUSED_LN", "1") != "0"
        self.device = torch.device(device) if device is not None else torch.device("cuda", gpu_id)
        if dtype not in _TORCH_DTYPES:
            raise ValueError(f"dtype must be one of {sorted(_TORCH_DTYPES)}")
        self.tdt = getattr(torch, _TORCH_DTYPES[dtype])
        if model is None:
            if model_name_or_path and os.path.isdir(model_name_or_path):
                from transformers import AutoModelForSequenceClassification, AutoTokenizer

                model = AutoModelForSequenceClassification.from_pretrained(model_name_or_path, local_files_only=True)
                tokenizer = tokenizer or AutoTokenizer.from_pretrained(model_name_or_path, local_files_only=True)
            elif model_name_or_path:
                raise FileNotFoundError(f"{model_name_or_path!r} is not a local model directory (no downloads)")
            else:
                model = build_random_cross_encoder(preset, seed)
        self.tokenizer = tokenizer if tokenizer is not None else HashWordTokenizer(
            getattr(getattr(model, "config", None), "vocab_size", 30522))
        self.model = model.to(self.device, self.tdt).eval()
        # K8: fused residual add + LayerNorm in every encoder layer (HIPRAG_FUSED_LN=0: PyTorch's two kernels)
        self.fused_layers = fuse_encoder_layers(self.model) if (fused_layernorm and self.device.type == "cuda") else 0
        max_pos = getattr(getattr(model, "config", None), "max_position_embeddings", None)
        self.max_length = min(int(max_length), int(max_pos)) if max_pos else int(max_length)
        self.batch_size = int(batch_size)
        if self.batch_size < 1:
            raise ValueError("batch_size must be at least one")
        self._cache: dict[str, list[int]] = {}
        self._cache_size = int(cache_size)
        self.model_name = model_name_or_path or f"random-init {preset}"

    # ------------------------------------------------------------------ tokens
    def _text_ids(self, text: str, cache: bool) -> list[int]:
        ids = self._cache.get(text) if cache else None
        if ids is None:
            ids = self.tokenizer(text, add_special_tokens=False, truncation=True,
                                 max_length=self.max_length)["input_ids"]
            if cache:
                if len(self._cache) >= self._cache_size:
                    self._cache.clear()
                self._cache[text] = ids
        return ids

    def warm(self, passages) -> int:
        """Tokenise passages into the cache ahead of reranking (e.g. at ingest, where the chunk text is
        tokenised for the embedder anyway); returns the number of newly cached passages."""
        before = len(self._cache)
        for p in passages:
            self._text_ids(p, cache=True)
        return len(self._cache) - before

    def _pair(self, q_ids: list[int], p_ids: list[int], passage_is_empty: bool = False
              ) -> tuple[list[int], list[int]]:
        cls_id = getattr(self.tokenizer, "cls_token_id", 101)
        sep_id = getattr(self.tokenizer, "sep_token_id", 102)
        if passage_is_empty:  # an empty pair text is no pair at all (Hugging Face: text_pair="" -> single)
            a = list(q_ids[: max(0, self.max_length - 2)])
            return [cls_id, *a, sep_id], [0] * (len(a) + 2)
        a, b = truncate_pair(q_ids, p_ids, self.max_length)
        ids = [cls_id, *a, sep_id, *b, sep_id]
        types = [0] * (len(a) + 2) + [1] * (len(b) + 1)
        return ids, types

    # ------------------------------------------------------------------ scoring
    def score_pairs(self, queries: list[str], passages: list[list[str]]):
        """Relevance (sigmoid of the cross-encoder logit) of every (query, passage) pair, as a list of
        float32 device tensors, one per query."""
        torch = self.torch
        pairs = []  # (query index, passage index, ids, types)
        for qi, (q, ps) in enumerate(zip(queries, passages)):
            q_ids = self._text_ids(q, cache=False)
            for pi, p in enumerate(ps):
                ids, types = self._pair(q_ids, self._text_ids(p, cache=True), passage_is_empty=not p)
                pairs.append((qi, pi, ids, types))
        offs = [0]
        for ps in passages:
            offs.append(offs[-1] + len(ps))
        flat = torch.empty(offs[-1], dtype=torch.float32, device=self.device)
        order = sorted(range(len(pairs)), key=lambda i: -len(pairs[i][2]))  # length-sorted batches
        pad_id = getattr(self.tokenizer, "pad_token_id", 0) or 0
        with torch.inference_mode():
            for b0 in range(0, len(order), self.batch_size):
                sel = order[b0:b0 + self.batch_size]
                width = len(pairs[sel[0]][2])
                ids = np.full((len(sel), width), pad_id, dtype=np.int64)
                types = np.zeros((len(sel), width), dtype=np.int64)
                lens = np.empty(len(sel), dtype=np.int64)
                dst = np.empty(len(sel), dtype=np.int64)
                for row, i in enumerate(sel):
                    qi, pi, t_ids, t_types = pairs[i]
                    n = len(t_ids)
                    ids[row, :n] = t_ids
                    types[row, :n] = t_types
                    lens[row] = n
                    dst[row] = offs[qi] + pi
                mask = (np.arange(width)[None, :] < lens[:, None]).astype(np.int64)
                logits = self.model(input_ids=torch.from_numpy(ids).to(self.device, non_blocking=True),
                                    attention_mask=torch.from_numpy(mask).to(self.device, non_blocking=True),
                                    token_type_ids=torch.from_numpy(types).to(self.device, non_blocking=True)).logits
                flat[torch.from_numpy(dst).to(self.device)] = torch.sigmoid(logits[:, 0].float())
        return [flat[offs[i]:offs[i + 1]] for i in range(len(queries))]

    def _select(self, scores: list, top_ns: list[int]) -> list[list[tuple[int, float]]]:
        """Per query: (position, relevance) of the top_n pairs, (relevance desc, position asc), on the GPU."""
        torch = self.torch
        out: list[list[tuple[int, float]]] = [[] for _ in scores]
        todo = [i for i, s in enumerate(scores) if len(s) and top_ns[i] > 0]
        if not todo:
            return out
        m = max(top_ns[i] for i in todo)
        offs = [0]
        for i in todo:
            offs.append(offs[-1] + len(scores[i]))
        rec = torch.empty((offs[-1], 2), dtype=torch.float64, device=self.device)
        for j, i in enumerate(todo):
            rec[offs[j]:offs[j + 1], 0] = scores[i].double()
            rec.view(torch.int64)[offs[j]:offs[j + 1], 1] = torch.arange(len(scores[i]), device=self.device)
        seg = torch.tensor(offs, dtype=torch.int64, device=self.device)
        top = torch.empty((len(todo), m, 2), dtype=torch.float64, device=self.device)
        _native.topk_records(rec.data_ptr(), len(todo), m, top.data_ptr(), seg_off_ptr=seg.data_ptr(),
                             stream=torch.cuda.current_stream(self.device).cuda_stream)
        pos = top.view(torch.int64)[..., 1].cpu().tolist()
        val = top[..., 0].cpu().tolist()
        for j, i in enumerate(todo):
            n = min(top_ns[i], len(scores[i]))
            out[i] = [(pos[j][t], val[j][t]) for t in range(n)]
        return out

    # ------------------------------------------------------------------ BaseReranker
    def rerank_batch(self, queries: list[str], results: list[list[RetrievalResult]],
                     top_k: int | None = None) -> list[list[RetrievalResult]]:
        """Rerank many queries' results in shared forward batches (same per-query output as rerank)."""
        top_ns = [min(top_k or len(r), len(r)) for r in results]
        scores = self.score_pairs(queries, [[r.chunk.content for r in rs] for rs in results])
        picks = self._select(scores, top_ns)
        return [[RetrievalResult(chunk=rs[p].chunk, score=float(s), rank=n + 1) for n, (p, s) in enumerate(pk)]
                for rs, pk in zip(results, picks)]

    async def rerank(self, query: str, results: list[RetrievalResult], top_k: int | None = None
                     ) -> list[RetrievalResult]:
        if not results:
            return results
        top_k = top_k or len(results)
        try:
            out = self.rerank_batch([query], [results], top_k)[0]
            logger.info(f"Reranked {len(results)} results to top {len(out)} using {self.model_name}")
            return out
        except Exception as e:  # the reference falls back to the retrieval order (openai_reranker.py:117-121)
            logger.error(f"Reranking failed: {e}")
            return results[:top_k]


class RerankerFactory:
    """Mirror of utu/rag/rerankers/factory.py:15-130 with the in-process backend added.

    ``"rocm"`` (aliases ``"local"``, ``"huggingface"``) builds TorchRocmReranker.  The reference's
    HTTP backends (auto / openai / service / tione / jina) are remote calls with no in-tree arithmetic
    and stay outside hiprag: they raise NotImplementedError after the reference's own argument checks
    (unknown backend -> ValueError, missing URL -> ValueError)."""

    @staticmethod
    def create(backend: str = "auto", **kwargs) -> BaseReranker:
        if backend in ("rocm", "local", "huggingface"):
            return TorchRocmReranker(**kwargs)
        if backend == "auto":
            if not os.getenv("UTU_RERANKER_URL"):
                raise ValueError("Could not auto-detect reranker configuration. "
                                 "Please set UTU_RERANK_URL environment variable.")
        elif backend in ("service", "tione"):
            if not (kwargs.get("service_url") or os.getenv("UTU_RERANKER_URL")):
                raise ValueError(f"service_url is required for {backend} reranker.")
        elif backend not in ("openai", "jina"):
            raise ValueError(f"Unknown reranker backend: {backend}. "
                             f"Supported backends: auto, openai, service, tione, jina, rocm")
        raise NotImplementedError(f"the HTTP reranker backend {backend!r} is outside the hiprag hot path; "
                                  "use backend='rocm' for the in-process MI355X cross-encoder")

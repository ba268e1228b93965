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
                 fused_layernorm: bool | None = None, unpadded: bool | None = None, **_ignored):
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
        # the encoder over the real tokens of each pair only (hiprag.rag.encoder), fp16 / bf16 on the GPU
        from . import encoder as _enc

        base = getattr(self.model, "base_model", None)
        if unpadded is None:
            unpadded = _enc._ENV and self.device.type == "cuda" and self.tdt != torch.float32
        self.unpadded = _enc.UnpaddedEncoder(base) if (unpadded and base is not None and _enc.UnpaddedEncoder.supported(base)
                                                       and _enc.sequence_logits(self.model, None, probe=True)) else None
        max_pos = getattr(getattr(model, "config", None), "max_position_embeddings", None)
        self.max_length = min(int(max_length), int(max_pos)) if max_pos else int(max_length)
        self.batch_size = int(batch_size)
        if self.batch_size < 1:
            raise ValueError("batch_size must be at least one")
        self._cache: dict[str, list[int]] = {}
        self._cache_np: dict[str, np.ndarray] = {}
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
    def _np_ids(self, text: str) -> np.ndarray:
        """Cached token ids of a passage as an int64 array (the pair assembly below is vectorised)."""
        a = self._cache_np.get(text)
        if a is None:
            a = np.asarray(self._text_ids(text, cache=True), np.int64)
            if len(self._cache_np) >= self._cache_size:
                self._cache_np.clear()
            self._cache_np[text] = a
        return a

    @staticmethod
    def _pair_lengths(n1: np.ndarray, n2: np.ndarray, max_length: int):
        """truncate_pair's longest_first lengths, vectorised over pairs."""
        target = max(0, int(max_length) - 3)
        over = n1 + n2 > target
        if not over.any():
            return n1, n2
        a1, a2 = n1.copy(), n2.copy()
        swap = n1 > n2
        s1, s2 = np.where(swap, n2, n1), np.where(swap, n1, n2)
        t2 = np.where(s1 > target, s1, np.maximum(s1, target - s1))
        both = s1 + t2 > target
        t1 = np.where(both, target // 2, s1)
        t2 = np.where(both, target // 2 + target % 2, t2)
        a1 = np.where(over, np.where(swap, t2, t1), a1)
        a2 = np.where(over, np.where(swap, t1, t2), a2)
        return a1, a2

    def score_pairs(self, queries: list[str], passages: list[list[str]]):
        """Relevance (sigmoid of the cross-encoder logit) of every (query, passage) pair, as a list of
        float32 device tensors, one per query.

        Pairs are encoded [CLS] q [SEP] p [SEP] (token types 0 / 1, longest_first truncation; an empty
        passage is the single sequence [CLS] q [SEP]) and run in length-sorted batches.  The batch
        matrices are assembled with vectorised numpy from cached per-passage id arrays and staged in
        pinned memory, so the host builds batch i+1 while the GPU runs batch i."""
        torch = self.torch
        cls_id = getattr(self.tokenizer, "cls_token_id", 101)
        sep_id = getattr(self.tokenizer, "sep_token_id", 102)
        pad_id = getattr(self.tokenizer, "pad_token_id", 0) or 0
        q_arr = [np.asarray(self._text_ids(q, cache=False), np.int64) for q in queries]
        offs = [0]
        for ps in passages:
            offs.append(offs[-1] + len(ps))
        n = offs[-1]
        flat = torch.empty(n, dtype=torch.float32, device=self.device)
        if n == 0:
            return [flat[offs[i]:offs[i + 1]] for i in range(len(queries))]
        qi = np.repeat(np.arange(len(queries)), [len(ps) for ps in passages])
        p_arr = [self._np_ids(p) if p else np.zeros(0, np.int64) for ps in passages for p in ps]
        empty = np.fromiter((not p for ps in passages for p in ps), bool, n)
        nq = np.fromiter((len(q_arr[i]) for i in qi), np.int64, n)
        npass = np.fromiter((len(a) for a in p_arr), np.int64, n)
        n1, n2 = self._pair_lengths(nq, npass, self.max_length)
        n1 = np.where(empty, np.minimum(nq, max(0, self.max_length - 2)), n1)  # single sequence
        n2 = np.where(empty, 0, n2)
        total = np.where(empty, n1 + 2, n1 + n2 + 3)
        order = np.argsort(-total, kind="stable")  # length-sorted batches (longest first)
        pin = self.device.type == "cuda"
        outs = []
        with torch.inference_mode():
            for b0 in range(0, n, self.batch_size):
                sel = order[b0:b0 + self.batch_size]
                nb, W = len(sel), int(total[sel[0]])
                s1, s2, emp = n1[sel], n2[sel], empty[sel]
                col = np.arange(W)[None, :]
                ids = np.full((nb, W), pad_id, np.int64)
                ids[:, 0] = cls_id
                rows = np.arange(nb)
                # query tokens at columns 1 .. n1, passage tokens at n1 + 2 .. n1 + n2 + 1
                qr = np.repeat(rows, s1)
                qc = 1 + np.arange(int(s1.sum())) - np.repeat(np.cumsum(s1) - s1, s1)
                ids[qr, qc] = np.concatenate([q_arr[qi[j]][:k] for j, k in zip(sel, s1)]) if len(qr) else 0
                ids[rows, 1 + s1] = sep_id
                pr = np.repeat(rows, s2)
                pc = (np.repeat(s1, s2) + 2 + np.arange(int(s2.sum())) - np.repeat(np.cumsum(s2) - s2, s2))
                if len(pr):
                    ids[pr, pc] = np.concatenate([p_arr[j][:k] for j, k in zip(sel, s2)])
                has_b = ~emp
                ids[rows[has_b], (s1 + s2 + 2)[has_b]] = sep_id
                L = total[sel][:, None]
                mask = (col < L).astype(np.int64)
                types = ((col >= (s1 + 2)[:, None]) & (col < L) & has_b[:, None]).astype(np.int64)
                if self.unpadded is not None:  # real tokens only: packed on the host, one upload
                    from .encoder import first_tokens, sequence_logits

                    pk = self.unpadded.pack(ids, mask, types)
                    h = self.unpadded.forward_packed(pk)
                    logits = sequence_logits(self.model, first_tokens(h, pk.cu_host))
                else:
                    t_ids, t_mask, t_types = (torch.from_numpy(x) for x in (ids, mask, types))
                    if pin:
                        t_ids, t_mask, t_types = (t.pin_memory() for t in (t_ids, t_mask, t_types))
                    logits = self.model(input_ids=t_ids.to(self.device, non_blocking=pin),
                                        attention_mask=t_mask.to(self.device, non_blocking=pin),
                                        token_type_ids=t_types.to(self.device, non_blocking=pin)).logits
                outs.append(torch.sigmoid(logits[:, 0].float()))
            dst = torch.from_numpy(order)
            if pin:
                dst = dst.pin_memory()
            flat[dst.to(self.device, non_blocking=pin)] = torch.cat(outs)
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

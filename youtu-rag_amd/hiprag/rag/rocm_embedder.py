"""In-process PyTorch-ROCm embedder behind BaseEmbedder.

Replaces the reference's HTTP hop to its embedding server (ServiceEmbedder,
utu/rag/embeddings/service_embedder.py:73-177) with the server's own computation
run in this process (LLMEmbeddingModel, docs/content/docs/en/youtu-embedding/
deploying-locally.mdx:41-126):

* tokenise with padding=True, truncation=True, max_length, add_special_tokens=True
  (mdx:83-90); queries are prefixed with
  "Instruction: {query_instruction} \\nQuery:" and passages with "" (mdx:64-71, :118-126);
* transformer forward on the GPU (PyTorch-ROCm -- the only torch compute here);
* the first len(tokenizer(instruction)["input_ids"]) mask positions are zeroed --
  with add_special_tokens=True, so even the empty passage instruction masks the
  tokeniser's special tokens, as the reference does (mdx:98-107);
* masked mean-pool + F.normalize run as the K7 HIP kernel (hr_pool_normalize,
  mdx:75-79, :114-115) straight from the model's hidden-state tensor.

``embed_texts_device`` keeps the vectors on the GPU so the ingest path
(hiprag.rag.ingest) can hand them to the index without a host round trip.

No checkpoint can be downloaded here: ``model_name_or_path`` must be a local
directory (AutoModel/AutoTokenizer with local_files_only); without one a
random-init BERT of the named preset shape is built from a config object with a
seeded init, with the offline HashWordTokenizer below.
"""
from __future__ import annotations

import asyncio
import itertools
import os
import re
import threading
import zlib
from concurrent.futures import ThreadPoolExecutor

import numpy as np

from .. import _native
from .base import BaseEmbedder

DEFAULT_QUERY_INSTRUCTION = "Given a search query, retrieve passages that answer the question"

# BertConfig shapes of the models the reference configs name (bge-base 768-d,
# bge-large 1024-d).
PRESETS = {
    "bge-base": dict(hidden_size=768, num_hidden_layers=12, num_attention_heads=12, intermediate_size=3072),
    "bge-large": dict(hidden_size=1024, num_hidden_layers=24, num_attention_heads=16, intermediate_size=4096),
    "tiny": dict(hidden_size=256, num_hidden_layers=2, num_attention_heads=4, intermediate_size=512),
}

_TORCH_DTYPES = {"float32": "float32", "fp32": "float32", "bfloat16": "bfloat16", "bf16": "bfloat16",
                 "float16": "float16", "fp16": "float16"}
_K7_DTYPE = {"float32": "f32", "bfloat16": "bf16", "float16": "f16"}
_PIN = os.environ.get("HIPRAG_EMBED_PIN", "1") != "0"  # A/B switch for the pinned token staging


# batches of ASCII texts go through the host text kernel (hr_hash_words; same ids), the rest through re + zlib
_NATIVE_TOK = os.environ.get("HIPRAG_NATIVE_TOKENIZER", "1") != "0"


class HashWordTokenizer:
    """Deterministic offline tokenizer for random-init models (no vocab files exist offline).

    Lower-cased words and punctuation marks (``\\w+|[^\\w\\s]``) hash (crc32) into
    [first_id, vocab_size); BERT's special ids ([PAD]=0, [CLS]=101, [SEP]=102).  The
    call signature and padding/truncation behaviour are the subset of Hugging Face's
    tokenizer __call__ the embedder uses: right padding to the longest sequence,
    truncation to max_length counting the special tokens, lists or "pt" tensors.
    """

    pad_token_id, cls_token_id, sep_token_id, first_id = 0, 101, 102, 1000
    _word = re.compile(r"\w+|[^\w\s]", re.UNICODE)

    _cache_max = 1 << 20  # words; cleared when full (ids are a pure function of the word)

    def __init__(self, vocab_size: int = 30522):
        self.vocab_size = int(vocab_size)
        self._cache: dict[str, int] = {}

    def _hash(self, w: str) -> int:
        if len(self._cache) >= self._cache_max:
            self._cache.clear()
        i = self._cache[w] = self.first_id + zlib.crc32(w.encode("utf-8")) % (self.vocab_size - self.first_id)
        return i

    def _ids(self, text: str) -> list[int]:
        words = self._word.findall(text.lower())
        ids = list(map(self._cache.get, words))  # C-speed lookups; misses come back as None
        if None in ids:
            ids = [self._hash(w) if i is None else i for w, i in zip(words, ids)]
        return ids

    def _native_batch(self, texts: list[str], cap, add_special_tokens: bool):
        """(flat ids, lengths) of all-ASCII texts from the host text kernel (hr_hash_words), else None."""
        if len(texts) < 8 or not all(t.isascii() for t in texts):
            return None
        data = "".join(texts).encode("ascii")
        offs = np.zeros(len(texts) + 1, np.int64)
        np.cumsum(np.fromiter(map(len, texts), np.int64, len(texts)), out=offs[1:])
        sp = add_special_tokens
        return _native.hash_words(data, offs, self.first_id, self.vocab_size - self.first_id,
                                  -1 if cap is None else cap, self.cls_token_id if sp else -1,
                                  self.sep_token_id if sp else -1)

    def __call__(self, text, padding=False, truncation=False, max_length=None, return_tensors=None,
                 add_special_tokens=True, **_):
        single = isinstance(text, str)
        texts = [text] if single else list(text)
        cap = max(0, int(max_length) - (2 if add_special_tokens else 0)) if truncation and max_length is not None \
            else None
        packed = self._native_batch(texts, cap, add_special_tokens) if return_tensors == "pt" and _NATIVE_TOK \
            else None
        seqs = []
        if packed is None:
            for t in texts:
                ids = self._ids(t)
                if cap is not None:
                    del ids[cap:]
                if add_special_tokens:
                    ids.insert(0, self.cls_token_id)
                    ids.append(self.sep_token_id)
                seqs.append(ids)
        if return_tensors == "pt":  # one (B, W) numpy fill, no nested-list tensor build
            import torch

            if packed is not None:
                flat, lens = packed
            else:
                lens = np.fromiter((len(s) for s in seqs), np.int64, len(seqs))
                flat = np.fromiter(itertools.chain.from_iterable(seqs), np.int64, int(lens.sum()))
            width = int(lens.max()) if padding and len(lens) else None
            if width is None and len(set(lens.tolist())) > 1:
                raise ValueError("return_tensors='pt' needs padding=True for ragged inputs")
            width = width if width is not None else (int(lens[0]) if len(lens) else 0)
            ids_np = np.full((len(lens), width), self.pad_token_id, np.int64)
            mask_np = np.arange(width)[None, :] < lens[:, None]
            ids_np[mask_np] = flat
            return {"input_ids": torch.from_numpy(ids_np), "attention_mask": torch.from_numpy(mask_np.astype(np.int64))}
        width = max((len(s) for s in seqs), default=0) if padding else None
        input_ids, mask = [], []
        for s in seqs:
            pad = (width - len(s)) if width is not None else 0
            input_ids.append(s + [self.pad_token_id] * pad)
            mask.append([1] * len(s) + [0] * pad)
        if single:
            return {"input_ids": input_ids[0], "attention_mask": mask[0]}
        return {"input_ids": input_ids, "attention_mask": mask}


def _fused_output_forward(self, hidden_states, input_tensor):
    """BertSelfOutput / BertOutput (and the XLM-R twins) with the residual add + LayerNorm as one
    HIP kernel (K8); dropout is the identity in eval mode."""
    ln = self.LayerNorm
    return _native.add_layernorm(self.dense(hidden_states), input_tensor, ln.weight, ln.bias, ln.eps)


def _fused_intermediate_forward(self, hidden_states):
    """BertIntermediate (and the XLM-R twin) with the exact GELU applied in place by hr_gelu_erf on the dense
    output (the bias is already in the GEMM's epilogue); torch's kernel where it does not apply."""
    h = self.dense(hidden_states)
    if _native.gelu_erf_(h) is None:
        h = self.intermediate_act_fn(h)
    return h


def fuse_encoder_layers(model) -> int:
    """Route every encoder layer's dense -> dropout -> LayerNorm(x + residual) block of a BERT /
    XLM-R model (modeling_bert.py BertSelfOutput / BertOutput) through K8, and, for half-precision models whose
    activation is the exact GELU (hidden_act "gelu"), the intermediate block's GELU through hr_gelu_erf.  Eval-mode
    models only.  Returns the number of blocks patched."""
    import types

    import torch

    n = 0
    p = next(model.parameters(), None)
    half = p is not None and p.dtype in (torch.float16, torch.bfloat16)
    exact_gelu = getattr(getattr(model, "config", None), "hidden_act", None) == "gelu"
    for m in model.modules():
        if type(m).__name__.endswith(("SelfOutput", "Output")) and hasattr(m, "dense") and hasattr(m, "LayerNorm") \
                and getattr(m.LayerNorm, "elementwise_affine", True):
            m.forward = types.MethodType(_fused_output_forward, m)
            n += 1
        elif half and exact_gelu and type(m).__name__.endswith("Intermediate") and hasattr(m, "dense") \
                and hasattr(m, "intermediate_act_fn") and type(m.intermediate_act_fn).__name__ == "GELUActivation":
            m.forward = types.MethodType(_fused_intermediate_forward, m)
            n += 1
    return n


def build_random_bert(preset: str = "bge-large", seed: int = 0, **overrides):
    """Seeded random-init BertModel of a named shape (no weights exist offline)."""
    import torch
    from transformers import BertConfig, BertModel

    cfg = dict(PRESETS[preset])
    cfg.update(overrides)
    config = BertConfig(vocab_size=30522, max_position_embeddings=512, **cfg)
    fork = torch.random.fork_rng(devices=[])
    with fork:
        torch.manual_seed(seed)
        model = BertModel(config, add_pooling_layer=False)
    return model


TUNED_GEMMS = os.path.join(os.path.dirname(os.path.abspath(__file__)), "tunableop_gfx950.csv")


def enable_tuned_gemms(path: str = TUNED_GEMMS) -> bool:
    """Use the TunableOp GEMM results shipped for gfx950 (opt-in: TorchRocmEmbedder(tuned_gemms=True)).  TunableOp is
    process-wide state, so this leaves an application's own setup alone: if TunableOp is already enabled, or any
    PYTORCH_TUNABLEOP_* variable is set, nothing is changed and False is returned.  Otherwise the results are read
    (their validators -- torch, HIP, hipBLASLt, rocBLAS versions and the GPU arch -- must match this process),
    tuning stays off, nothing is written on exit (the shipped file is never rewritten, no temp file is left), and
    TunableOp is enabled only if the results were accepted.  Returns whether they were."""
    import torch

    if not (os.path.exists(path) and torch.cuda.is_available()):
        return False
    import torch.cuda.tunable as tun

    if tun.is_enabled() or any(k.startswith("PYTORCH_TUNABLEOP_") for k in os.environ):
        return False
    tun.tuning_enable(False)  # (TunableOp writes its results file at exit only while tuning is enabled)
    if hasattr(tun, "write_file_on_exit"):  # (newer torch: say so explicitly)
        tun.write_file_on_exit(False)
    ok = bool(tun.read_file(path))
    if ok:
        tun.enable(True)
    return ok


class _LoopQueue:
    """One event loop's waiting queries and whether its drain task is running."""

    __slots__ = ("pending", "running", "__weakref__")

    def __init__(self):
        self.pending: list = []
        self.running = False


class _QueryCoalescer:
    """Concurrent ``embed_query`` calls as ONE forward: the reference embeds per call (VectorRetriever.retrieve,
    base_retriever.py:57, one HTTP request each), so N concurrent retrievals were N one-query forwards run on the
    event loop, each blocking it.  Here a call queues its query and awaits its own future (so a caller's
    cancellation cancels only its query); a drain task takes up to ``max_batch`` waiting queries per forward and
    runs it in one worker thread (the GPU wait and the host list conversion off the loop), one batch at a time
    while the next one gathers.  Each vector is the one ``encode_queries`` gives for that query (rows are
    independent through the encoder; a different batch size can only change GEMM rounding).

    Every event loop has its own queue and drain (asyncio futures are not thread-safe: a drain only ever resolves
    its own loop's futures, on that loop); the loops share the one worker thread, so forwards still run one at a
    time.  A loop that is closed leaves its queue behind with it."""

    def __init__(self, emb, max_batch: int):
        import weakref

        self.emb, self.max_batch = emb, max(1, int(max_batch))
        self._queues: "weakref.WeakKeyDictionary" = weakref.WeakKeyDictionary()  # loop -> _LoopQueue
        self._qlock = threading.Lock()
        self.forwards = 0  # diagnostics: forwards run / queries embedded through them
        self.queries = 0
        self._pool = None
        self._pool_lock = threading.Lock()

    def _queue(self, loop) -> _LoopQueue:
        with self._qlock:
            lq = self._queues.get(loop)
            if lq is None:
                lq = self._queues[loop] = _LoopQueue()
            return lq

    @property
    def pending(self) -> list:
        """The waiting queries of the calling thread's running loop (diagnostics / tests)."""
        try:
            loop = asyncio.get_running_loop()
        except RuntimeError:
            return []
        lq = self._queues.get(loop)
        return lq.pending if lq is not None else []

    def submit(self, query: str) -> asyncio.Future:
        loop = asyncio.get_running_loop()
        fut = loop.create_future()
        lq = self._queue(loop)
        lq.pending.append((query, fut))
        if not lq.running:
            lq.running = True
            # drain on the next loop iteration: every task that is ready now queues its query first
            loop.call_soon(lambda: loop.create_task(self._drain(lq)))
        return fut

    def _executor(self):
        with self._pool_lock:
            if self._pool is None:
                self._pool = ThreadPoolExecutor(max_workers=1, thread_name_prefix="hiprag-embed")
            return self._pool

    async def _drain(self, lq: _LoopQueue):
        loop = asyncio.get_running_loop()
        batch: list = []
        try:
            while lq.pending:
                batch, lq.pending = lq.pending[: self.max_batch], lq.pending[self.max_batch:]
                batch = [e for e in batch if not e[1].done()]  # (cancelled while waiting)
                if not batch:
                    continue
                try:
                    vecs = await loop.run_in_executor(self._executor(), self.emb._query_lists, [q for q, _ in batch])
                except Exception as exc:  # noqa: BLE001 -- this batch's callers see the failure
                    for _, f in batch:
                        if not f.done():
                            f.set_exception(exc)
                    batch = []
                    continue
                self.forwards += 1
                self.queries += len(batch)
                for (_, f), v in zip(batch, vecs):
                    if not f.done():
                        f.set_result(v)
                batch = []
        except BaseException as exc:  # the drain itself stopped (loop shutdown): no caller is left waiting
            err = exc if isinstance(exc, Exception) else RuntimeError(f"query embedding stopped: {exc!r}")
            for _, f in batch + lq.pending:
                if not f.done():
                    f.set_exception(err)
            lq.pending = []
            raise
        finally:
            lq.running = False

    def close(self):
        with self._pool_lock:
            if self._pool is not None:
                self._pool.shutdown(wait=True)
                self._pool = None


class TorchRocmEmbedder(BaseEmbedder):
    """BaseEmbedder running the embedding model in-process on an MI355X (provider "rocm")."""

    def __init__(self, model_name_or_path: str | None = None, *, model=None, tokenizer=None, preset: str = "bge-large",
                 batch_size: int = 64, max_length: int = 1024, gpu_id: int = 0, device=None, dtype: str = "float32",
                 query_instruction: str | None = DEFAULT_QUERY_INSTRUCTION, seed: int = 0,
                 trust_remote_code: bool = False, fused_layernorm: bool | None = None, unpadded: bool | None = None,
                 forward_tokens: int | None = None, cuda_graphs: bool | None = None,
                 tuned_gemms: bool | None = None, coalesce_queries: bool = True, **_ignored):
        import torch

        self.torch = torch
        if fused_layernorm is None:
            fused_layernorm = os.environ.get("HIPRAG_FUSED_LN", "1") != "0"
        self.device = torch.device(device) if device is not None else torch.device("cuda", gpu_id)
        if dtype not in _TORCH_DTYPES:
            raise ValueError(f"dtype must be one of {sorted(_TORCH_DTYPES)}")
        self.dtype_name = _TORCH_DTYPES[dtype]
        tdt = getattr(torch, self.dtype_name)
        if model is None:
            if model_name_or_path and os.path.isdir(model_name_or_path):
                from transformers import AutoModel, AutoTokenizer

                model = AutoModel.from_pretrained(model_name_or_path, local_files_only=True,
                                                  trust_remote_code=trust_remote_code)
                tokenizer = tokenizer or AutoTokenizer.from_pretrained(
                    model_name_or_path, padding_side="right", local_files_only=True,
                    trust_remote_code=trust_remote_code)
            elif model_name_or_path:
                raise FileNotFoundError(f"{model_name_or_path!r} is not a local model directory (no downloads)")
            else:
                model = build_random_bert(preset, seed)
        self.tokenizer = tokenizer if tokenizer is not None else HashWordTokenizer(
            getattr(getattr(model, "config", None), "vocab_size", 30522))
        self.model = model.to(self.device, tdt).eval()
        # encoder GEMMs from the TunableOp results shipped for gfx950 (tools/embed_tune.py: every hipBLASLt / rocBLAS
        # solution of the bge shapes at each 64-token count benchmarked, the fastest kept), read-only; shapes not in
        # the file, or a file whose library versions do not match, keep the heuristic choice.  Opt-in (TunableOp is
        # process-wide state): tuned_gemms=True, or HIPRAG_TUNED_GEMMS=1
        if tuned_gemms is None:
            tuned_gemms = os.environ.get("HIPRAG_TUNED_GEMMS", "0") == "1"
        tuned_gemms = bool(tuned_gemms) and self.device.type == "cuda" and self.dtype_name != "float32"
        self.tuned_gemms = enable_tuned_gemms() if tuned_gemms else False
        # K8: fused residual add + LayerNorm in every encoder layer (HIPRAG_FUSED_LN=0: PyTorch's two kernels)
        self.fused_layers = fuse_encoder_layers(self.model) if (fused_layernorm and self.device.type == "cuda") else 0
        # the encoder over the real tokens only (hiprag.rag.encoder): fp16 / bf16 models on the GPU, where the
        # varlen flash kernel serves the attention; fp32 keeps Hugging Face's padded forward (parity listings)
        from . import encoder as _enc

        if unpadded is None:
            unpadded = _enc._ENV and self.device.type == "cuda" and self.dtype_name != "float32"
        self.unpadded = _enc.UnpaddedEncoder(self.model) if (unpadded and _enc.UnpaddedEncoder.supported(self.model)) \
            else None
        # packed forwards up to 8192 tokens (query batches) replayed from HIP graphs (encoder.GraphedForward): their
        # ~300 kernel launches per forward, not the GPU, bound them; cuda_graphs=False runs them eagerly
        if cuda_graphs is None:
            cuda_graphs = self.unpadded is not None
        self.graphed = _enc.GraphedForward(self.unpadded) if (cuda_graphs and self.unpadded is not None) else None
        max_pos = getattr(getattr(model, "config", None), "max_position_embeddings", None)
        self.max_length = min(int(max_length), int(max_pos)) if max_pos else int(max_length)
        self.batch_size = int(batch_size)
        if self.batch_size < 1:
            raise ValueError("batch_size must be at least one")
        self.query_instruction = (f"Instruction: {query_instruction} \nQuery:" if query_instruction else "Query:")
        self.doc_instruction = ""
        self.dim = int(getattr(getattr(model, "config", None), "hidden_size", 0)) or None
        self._n_instr: dict[str, int] = {}  # instruction -> its token count (fixed per tokenizer)
        # unpadded forwards: consecutive tokenizer batches are packed into one forward of at least this
        # many tokens (bigger GEMMs; 0 = one forward per batch)
        if forward_tokens is None:
            forward_tokens = int(os.environ.get("HIPRAG_FORWARD_TOKENS", "0"))
        self.forward_tokens = max(0, int(forward_tokens))
        # forwards from more than one thread (the query coalescer's worker, ingest on the loop) take turns: the HIP
        # graphs' static inputs are shared (GPU order is the device's stream order either way)
        self._fwd_lock = threading.Lock()
        # concurrent embed_query calls share forwards of up to batch_size queries (False: one forward per call,
        # on the calling thread, as before)
        self._coalescer = _QueryCoalescer(self, self.batch_size) if coalesce_queries else None

    # ------------------------------------------------------------------ core
    def _n_instruction_tokens(self, instruction: str) -> int:
        n = self._n_instr.get(instruction)
        if n is None:
            n = self._n_instr[instruction] = len(self.tokenizer(instruction, padding=False, truncation=True,
                                                                max_length=self.max_length,
                                                                add_special_tokens=True)["input_ids"])
        return n

    def _pool(self, hidden, mask, n_instr: int):
        """K7: masked mean-pool + L2 normalise on the GPU -> (B, H) float32."""
        torch = self.torch
        B, T, H = hidden.shape
        out = torch.empty((B, H), dtype=torch.float32, device=hidden.device)
        _native.pool_normalize(hidden.data_ptr(), _K7_DTYPE[self.dtype_name], mask.data_ptr(), B, T, H, n_instr,
                               out.data_ptr(), torch.cuda.current_stream(hidden.device).cuda_stream)
        return out

    def encode(self, sentences: list[str], instruction: str):
        """One batch -> (B, H) float32 device tensor (LLMEmbeddingModel.encode, mdx:81-116)."""
        torch = self.torch
        inputs = self.tokenizer(list(sentences), padding=True, truncation=True, return_tensors="pt",
                                max_length=self.max_length, add_special_tokens=True)
        # pinned staging: the H2D copy is then truly asynchronous, so the host tokenises batch i+1
        # while the GPU runs batch i's forward (a pageable copy waits for the stream to drain)
        pin = self.device.type == "cuda" and _PIN
        n_instr = self._n_instruction_tokens(instruction)
        if self.unpadded is not None:  # real tokens only: packed on the host, one upload, packed K7
            return self._forward_packed([inputs], n_instr)
        inputs = {k: (v.pin_memory() if pin else v).to(self.device, non_blocking=True) for k, v in inputs.items()}
        with self._fwd_lock, torch.inference_mode():
            hidden = self.model(**inputs)[0]
            if hidden.dtype != getattr(torch, self.dtype_name):
                hidden = hidden.to(getattr(torch, self.dtype_name))
            hidden = hidden.contiguous()
            mask = inputs["attention_mask"].to(torch.int32).contiguous()
            return self._pool(hidden, mask, n_instr)

    def _forward_packed(self, batches: list, n_instr: int):
        """Unpadded forward of one or more tokenizer batches as ONE packed batch -> (sum B, H) float32."""
        torch = self.torch
        with self._fwd_lock, torch.inference_mode():
            gf = self.graphed
            ntok = sum(int(b["attention_mask"].sum()) for b in batches)
            if gf is not None and ntok + gf.granule > gf.max_tokens:
                gf = None
            pk = self.unpadded.pack([b["input_ids"] for b in batches], [b["attention_mask"] for b in batches],
                                    [b.get("token_type_ids") for b in batches], granule=gf.granule if gf else 0)
            hidden = gf(pk) if gf is not None else self.unpadded.forward_packed(pk)
            if hidden.dtype != getattr(torch, self.dtype_name):
                hidden = hidden.to(getattr(torch, self.dtype_name))
            hidden = hidden.contiguous()
            B, H = len(pk.lengths), hidden.shape[-1]
            out = torch.empty((B, H), dtype=torch.float32, device=hidden.device)
            _native.pool_normalize_packed(hidden.data_ptr(), _K7_DTYPE[self.dtype_name], pk.cu.data_ptr(), B, H,
                                          n_instr, out.data_ptr(), torch.cuda.current_stream(hidden.device).cuda_stream)
            return out

    def _encode_packs(self, texts: list[str], order: list[int], instruction: str) -> list:
        """Unpadded path over many batches: tokenizer batches of batch_size (in `order`) gathered into
        forwards of >= forward_tokens real tokens."""
        n_instr = self._n_instruction_tokens(instruction)
        outs, group, tok = [], [], 0
        for i in range(0, len(texts), self.batch_size):
            b = self.tokenizer([texts[j] for j in order[i:i + self.batch_size]], padding=True, truncation=True,
                               return_tensors="pt", max_length=self.max_length, add_special_tokens=True)
            group.append(b)
            tok += int(b["attention_mask"].sum())
            if tok >= self.forward_tokens:
                outs.append(self._forward_packed(group, n_instr))
                group, tok = [], 0
        if group:
            outs.append(self._forward_packed(group, n_instr))
        return outs

    def _encode_all(self, texts: list[str], prefix: str, instruction: str):
        torch = self.torch
        texts = [f"{prefix}{t}" for t in texts]
        if len(texts) <= self.batch_size:  # one batch: the caller's order (padding is the same either way)
            if not texts:
                return torch.empty((0, self.dim or 0), dtype=torch.float32, device=self.device)
            return self.encode(texts, instruction)
        # several batches: length-sorted (character count as the token-count proxy), so each batch
        # pads to about its own length instead of the longest text of a random mix; rows are
        # independent through the encoder, so only the order of the output rows changes back
        order = sorted(range(len(texts)), key=lambda i: len(texts[i]))
        # the permutation goes up first, asynchronously from pinned memory: a pageable copy after the
        # forwards would wait for all of them (the host then could not tokenise the next pack meanwhile)
        perm = torch.as_tensor(order, dtype=torch.int64)
        if self.device.type == "cuda" and _PIN:
            perm = perm.pin_memory()
        perm = perm.to(self.device, non_blocking=True)
        if self.unpadded is not None and self.forward_tokens > 0:
            parts = self._encode_packs(texts, order, instruction)
        else:
            parts = [self.encode([texts[j] for j in order[i:i + self.batch_size]], instruction)
                     for i in range(0, len(texts), self.batch_size)]
        out = torch.empty((len(texts), parts[0].shape[1]), dtype=torch.float32, device=self.device)
        out[perm] = torch.cat(parts)
        return out

    def encode_queries(self, queries):
        queries = queries if isinstance(queries, list) else [queries]
        return self._encode_all(queries, self.query_instruction, self.query_instruction)

    def encode_passages(self, passages):
        passages = passages if isinstance(passages, list) else [passages]
        return self._encode_all(passages, self.doc_instruction, self.doc_instruction)

    # ------------------------------------------------------------- BaseEmbedder
    def embed_texts_device(self, texts: list[str]):
        """Passages -> (n, H) float32 device tensor (no host copy; used by the GPU ingest path)."""
        return self.encode_passages(list(texts))

    def embed_queries_device(self, queries: list[str]):
        return self.encode_queries(list(queries))

    async def embed_texts(self, texts: list[str]) -> list[list[float]]:
        return self.encode_passages(list(texts)).cpu().tolist()

    def _query_lists(self, queries: list[str]) -> list[list[float]]:
        return self.encode_queries(list(queries)).cpu().numpy().tolist()

    async def embed_query(self, query: str) -> list[float]:
        if self._coalescer is None:
            return self.encode_queries([query])[0].cpu().tolist()
        return await self._coalescer.submit(query)

    async def embed_queries(self, queries: list[str]) -> list[list[float]]:
        return self.encode_queries(list(queries)).cpu().tolist()

"""IVF-flat candidate generation on the HIP index (BASELINE.json configs[4]: "50M×1024 fp16 ANN
candidate-gen + cross-encoder rerank top-100").

The reference has no ANN index of its own: its production store is Chroma's HNSW
(chroma_store.py:41-59, approximate, third-party).  This is the MI355X replacement for that
approximate stage: an inverted-file index whose lists are stored in the same 32-row MFMA tile
layout as the exact index (one ``NativeIndex`` holds the rows in list order, every list starting
on a tile; pad rows are dead), searched by ``hr_ivf_search`` (youtu-rag_amd/csrc/hr_ivf.hip):

  * coarse stage: exact canonical fp64 scores of every centroid, top-``nprobe`` lists per query;
  * list stage: exact canonical fp64 scores of every row of the probed lists, top-k per query.

Results are therefore *exact within the probed lists* (bit-identical to the oracle's restatement,
tests/test_gpu_ivf.py); recall against the full exact search is the ANN trade-off, and
``nprobe = nlist`` is the exact search.  Each probed tile is read once per query, so a batch reads
about ``B * nprobe / nlist`` of the corpus instead of all of it.

Training (spherical k-means for cosine, max-inner-product k-means for dot) and list assignment
are build-time GEMMs and run through PyTorch (hipBLASLt); only the search is on the query path.
Multi-GPU: every rank holds its row shard's share of every list (shared centroids), returns its
exact top-k of its visible rows with bound -inf, and ``IvfShardedSearch`` merges them with the
same packed all-gather + merge as the exact search.
"""
from __future__ import annotations

import numpy as np

from . import _native
from .dist import ShardedSearch


def _round64(d: int) -> int:
    return (d + 63) // 64 * 64


class IvfIndex:
    """IVF-flat index of one shard on one GPU."""

    def __init__(self, dim: int, nlist: int, dtype: str = "f16", metric: str = "cosine", device: int = 0):
        import torch

        if metric not in ("cosine", "ip", "dot"):
            raise NotImplementedError("IVF lists support cosine and dot (inner product)")
        self.torch = torch
        self.dim, self.nlist, self.dtype = int(dim), int(nlist), dtype
        self.metric = "ip" if metric == "dot" else metric
        self.dev = torch.device("cuda", device)
        self.device = device
        self.dpad = _round64(self.dim)
        self.index = _native.NativeIndex(self.dim, dtype, self.metric, device)
        self.centroids = None      # (nlist, dpad) fp32, processed (unit norm for cosine)
        self.list_tiles = None     # (nlist + 1,) int64 tile offsets
        self.ids = None            # (positions,) int64 original id per stored position, -1 for pads
        self.max_list_tiles = 0
        self.n = 0

    # ---------------------------------------------------------------- build
    def _process(self, x):
        torch = self.torch
        x = x.to(torch.float32)
        if self.metric == "cosine":
            x = torch.nn.functional.normalize(x, dim=1)
        return x

    def train(self, sample, iters: int = 10, seed: int = 0):
        """k-means on a (m, dim) fp32 device sample: spherical for cosine, max-inner-product with
        unit centroids for dot.  Empty lists keep their previous centroid."""
        torch = self.torch
        x = self._process(sample.to(self.dev))
        m = x.shape[0]
        if m < self.nlist:
            raise ValueError(f"training sample ({m}) smaller than nlist ({self.nlist})")
        g = torch.Generator(device=self.dev)
        g.manual_seed(int(seed))
        cent = x[torch.randperm(m, generator=g, device=self.dev)[: self.nlist]].clone()
        cent = torch.nn.functional.normalize(cent, dim=1)
        for _ in range(iters):
            assign = self._assign(x, cent)
            sums = torch.zeros_like(cent).index_add_(0, assign, x)
            cnt = torch.bincount(assign, minlength=self.nlist)
            upd = cnt > 0
            cent[upd] = torch.nn.functional.normalize(sums[upd], dim=1)
        c = torch.zeros((self.nlist, self.dpad), dtype=torch.float32, device=self.dev)
        c[:, : self.dim] = cent
        self.centroids = c.contiguous()
        return self

    def _assign(self, x, cent, chunk: int = 1 << 16):
        torch = self.torch
        out = torch.empty(x.shape[0], dtype=torch.int64, device=self.dev)
        for i in range(0, x.shape[0], chunk):
            out[i:i + chunk] = torch.argmax(x[i:i + chunk] @ cent.T, dim=1)
        return out

    def build(self, n: int, rows, id_offset: int = 0, chunk: int = 1 << 18):
        """Bulk build from ``rows(i0, i1) -> (i1 - i0, dim) fp32 device tensor`` (raw vectors; the
        store normalises for cosine).  Two passes: list assignment, then placement by list."""
        torch = self.torch
        if self.centroids is None:
            raise RuntimeError("train() the coarse quantizer first")
        if self.n:
            raise RuntimeError("IVF lists are built once (bulk); create a new index to rebuild")
        cent = self.centroids[:, : self.dim]
        lists = torch.empty(n, dtype=torch.int64, device=self.dev)
        for i in range(0, n, chunk):
            lists[i:i + chunk] = self._assign(self._process(rows(i, min(n, i + chunk))), cent)
        counts = torch.bincount(lists, minlength=self.nlist)
        tiles = (counts + 31) // 32
        list_tiles = torch.zeros(self.nlist + 1, dtype=torch.int64, device=self.dev)
        list_tiles[1:] = torch.cumsum(tiles, 0)
        order = torch.sort(lists, stable=True).indices          # rows grouped by list, row order inside
        first = torch.zeros(self.nlist, dtype=torch.int64, device=self.dev)
        first[1:] = torch.cumsum(counts, 0)[:-1]
        rank = torch.arange(n, dtype=torch.int64, device=self.dev) - first[lists[order]]
        dest = torch.empty(n, dtype=torch.int64, device=self.dev)
        dest[order] = list_tiles[lists[order]] * 32 + rank
        total = int(list_tiles[-1].item()) * 32
        self.index.reserve(total)
        stream = torch.cuda.current_stream(self.dev).cuda_stream
        for i in range(0, n, chunk):
            j = min(n, i + chunk)
            x = rows(i, j).to(torch.float32).contiguous()
            d = dest[i:j].contiguous()
            self.index.add_device_at(x.data_ptr(), j - i, d.data_ptr(), total, stream=stream)
        ids = torch.full((max(total, 1),), -1, dtype=torch.int64, device=self.dev)
        ids[dest] = torch.arange(n, dtype=torch.int64, device=self.dev) + int(id_offset)
        self.ids, self.list_tiles = ids, list_tiles
        self.max_list_tiles = int(tiles.max().item()) if n else 0
        self.n = n
        self.lists_of_rows = lists  # row -> list (tests, the oracle restatement)
        return self

    def build_synthetic(self, seed: int, row0: int, n: int, chunk: int = 1 << 18):
        """Build from the counter-based synthetic corpus rows [row0, row0 + n) (ids = global rows)."""
        torch = self.torch
        stream = lambda: torch.cuda.current_stream(self.dev).cuda_stream  # noqa: E731

        def rows(i0, i1):
            x = torch.empty((i1 - i0, self.dim), dtype=torch.float32, device=self.dev)
            _native.gen_rows_device(seed, row0 + i0, i1 - i0, self.dim, x.data_ptr(), stream())
            return x

        return self.build(n, rows, id_offset=row0, chunk=chunk)

    def list_members(self) -> list[np.ndarray]:
        """Original ids of every list (host; tests and diagnostics)."""
        lt = self.list_tiles.cpu().numpy()
        ids = self.ids.cpu().numpy()
        return [ids[lt[l] * 32: lt[l + 1] * 32][ids[lt[l] * 32: lt[l + 1] * 32] >= 0] for l in range(self.nlist)]

    # ---------------------------------------------------------------- search
    def search_candidates(self, q, k: int, nprobe: int, cand, bound, probes=None, mask_ptr: int = 0, stream=None):
        """Exact top-k of the probed lists' rows for a (B, dim) fp32 device batch, as B*k candidate
        records (score, global id) + bounds (all -inf), on ``stream`` (default: current)."""
        torch = self.torch
        if self.ids is None:
            raise RuntimeError("build() the index first")
        st = stream if stream is not None else torch.cuda.current_stream(self.dev).cuda_stream
        q = q.contiguous()
        self.index.ivf_search(self.centroids.data_ptr(), self.nlist, self.list_tiles.data_ptr(), self.max_list_tiles,
                              self.ids.data_ptr(), q.data_ptr(), q.shape[0], nprobe, k, cand.data_ptr(),
                              bound.data_ptr(), 0 if probes is None else probes.data_ptr(), mask_ptr, st)

    def search(self, q, k: int, nprobe: int):
        """(scores (B, k) fp32, ids (B, k) int64) device tensors; -inf / -1 padding."""
        torch = self.torch
        B = q.shape[0]
        cand = torch.empty((B, k, 2), dtype=torch.float64, device=self.dev)
        bound = torch.empty(B, dtype=torch.float64, device=self.dev)
        self.search_candidates(q, k, nprobe, cand, bound)
        s = cand[..., 0].to(torch.float32)
        r = cand.view(torch.int64)[..., 1].clone()
        return s, r

    def close(self):
        self.index.close()


class IvfShardedSearch(ShardedSearch):
    """Row-sharded IVF over the ranks (shared centroids): each rank's exact top-k of its visible
    rows, one packed all-gather, the exact merge.  Bounds are -inf, so no fallback ever runs."""

    def __init__(self, ivf: IvfIndex, max_batch: int, k: int, nprobe: int, group=None, depth: int = 2):
        super().__init__(ivf.index, 0, max_batch, kc=k, group=group, device=ivf.dev, depth=depth, overlap=False)
        self.ivf, self.nprobe = ivf, int(nprobe)

    def _shard_search(self, q, k, cand, bound, mask_ptr):
        self.ivf.search_candidates(q, self.kc, self.nprobe, cand, bound, mask_ptr=mask_ptr, stream=self._stream())

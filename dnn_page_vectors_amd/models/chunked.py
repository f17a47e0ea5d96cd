"""Long-page chunked encoder (BASELINE config 5: "Long-page 4k-token chunked encoder,
mean-pool, fp8 MFMA on CDNA4").

The reference scales to long pages only by truncation + a global max-pool
(data_utils.py:29-68, cnn_dssm_th.py:94).  Here a page of up to
``num_chunks * chunk_len`` (8 x 512 = 4096) hashed trigram ids is cut into chunks,
every chunk is encoded independently by the DSSM MLP tower (bag-of-trigrams via the
counts GEMM — with ``use_fp8`` e4m3 counts x e4m3 table on the block-scaled fp8 MFMA,
csrc/kernels/gemm_mx8.hip — then fp8 e4m3 MFMA dense layers), and the page vector is the MEAN of its
non-empty chunk vectors (empty = all padding; masked out).  Chunks are independent, so
a page could be split over CUs or GPUs with one all-reduce of partial sums (the
"context parallel" of this workload) — at 288 GB per MI355X it is not
needed.  Queries use the same tower type without chunking.

``chunk_encoder`` selects the per-chunk encoder ("encode each chunk (CDSSM or
MLP or BERT)"):
* ``"mlp"``   — the DSSM MLP tower above (config 5 as benchmarked; fp8 e4m3 dense layers
  with ``use_fp8``);
* ``"cdssm"`` — the reference's conv tower (cnn_dssm_th.py:83-139) on every chunk through
  the fused gather -> dropout -> conv -> max-pool HIP kernel (the N x C chunks are the
  kernel's samples; each chunk max-pools over its own windows), then Dense + ReLU;
  chunk vectors mean-pooled as above (``chunk_pool='mean'``, the default).  ``chunk_pool='max'``
  instead takes the element-wise max of the chunks' pooled conv features before ONE Dense +
  ReLU — exactly the reference's global max-pool over all windows of the page
  (cnn_dssm_th.py:94) for pages of up to num_chunks x chunk_len tokens — but it learns slower
  in the 500-step quality protocol (Recall@10 0.13 vs 0.22 for the mean, lr 3e-3; the max
  routes each feature's gradient to one chunk: profiles/r4_quality/README.md).  Needs the
  CDSSM geometry (embedding_dim <= 104, filters (3, 4) x 150): preset ``longpage_cdssm``.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from ..ops import dense as dops
from .base import TwoTowerModel
from ..ops import conv_pool as cops
from .cdssm import CDSSMTower
from .mlp_dssm import MLPTower


class ChunkedPageEncoder(TwoTowerModel):
    def __init__(self, cfg, vocab_size: int):
        super().__init__(cfg)
        gen = torch.Generator().manual_seed(int(cfg.seed))
        act = getattr(cfg, "mlp_act", "tanh")
        self.vocab_size = vocab_size
        self.chunk_len = int(cfg.chunk_len)
        self.num_chunks = int(cfg.num_chunks)
        self.encoder = getattr(cfg, "chunk_encoder", "mlp")
        pool = getattr(cfg, "chunk_pool", "auto")
        self.chunk_pool = "mean" if pool == "auto" else pool
        if self.chunk_pool not in ("mean", "max") or (self.chunk_pool == "max" and self.encoder != "cdssm"):
            raise ValueError(f"chunk_pool={pool!r}: 'mean', or 'max' with chunk_encoder='cdssm'")
        if self.encoder == "cdssm":
            if cfg.use_fp8:
                raise ValueError("chunk_encoder='cdssm' runs the bf16 conv kernel: set use_fp8=False")
            self.query_tower = CDSSMTower(vocab_size, cfg, gen)
            self.doc_towers = nn.ModuleList([CDSSMTower(vocab_size, cfg, gen)])
        else:
            self.query_tower = MLPTower(vocab_size, cfg.mlp_dims, act, gen, use_fp8=cfg.use_fp8)
            self.doc_towers = nn.ModuleList([MLPTower(vocab_size, cfg.mlp_dims, act, gen, use_fp8=cfg.use_fp8)])
            self.doc_towers[0].long_bags = True  # chunk bags: the counts plan (fp8 MFMA with use_fp8)

    @property
    def out_dim(self) -> int:
        return self.cfg.hidden_dims if self.encoder == "cdssm" else self.cfg.mlp_dims[-1]

    def bf16_mirror_params(self):
        if self.encoder == "cdssm":
            return []  # the conv tower casts its bf16 table copy in build_cache
        return [n for n, _ in self.named_parameters() if n.endswith(".embedding")]

    def build_cache(self):
        if not self.query_tower.embedding.is_cuda:
            return {}
        q, d = self.query_tower, self.doc_towers[0]
        if self.encoder == "cdssm" and cops.PREP_MULTI and q.build_cache_ok() and d.build_cache_ok():
            res = cops.prep_towers([(t.embedding.detach(), t.conv_w[0].detach(), t.conv_w[1].detach())
                                    for t in (q, d)])
            return {"query": res[0], "doc0": res[1]}
        return {"query": q.build_cache(), "doc0": d.build_cache()}

    def _tower(self, t, ids, training, seed, cache):
        if self.encoder == "cdssm":
            return t(ids, training, seed, cache)
        return t(ids, cache)

    def tower_forward(self, tower: str, ids: torch.Tensor, training: bool, seed: int, slot: int = 0) -> torch.Tensor:
        cache = self.compute_cache()
        if tower == "query":
            return self._tower(self.query_tower, ids, training, seed, cache.get("query"))
        N, L = ids.shape
        C = max(1, -(-L // self.chunk_len))
        pad = C * self.chunk_len - L
        if pad:
            ids = torch.nn.functional.pad(ids, (0, pad))
        chunks = ids.reshape(N * C, self.chunk_len)
        if self.encoder == "cdssm" and self.chunk_pool == "max":
            t = self.doc_towers[0]
            f = t.features(chunks, training, seed, cache.get("doc0")).view(N, C, -1)
            # empty chunks (all padding) must not win the max: their features -> 0 (every
            # real feature is a ReLU output >= 0)
            live = (ids.view(N, C, self.chunk_len) != 0).any(dim=2, keepdim=True)
            f = torch.where(live, f, torch.zeros((), dtype=f.dtype, device=f.device))
            return t.head(f.amax(dim=1), training)
        v = self._tower(self.doc_towers[0], chunks, training, seed, cache.get("doc0")).view(N, C, -1)
        # masked mean over the non-empty chunks (one fused HIP kernel per direction on GPU)
        return dops.chunk_mean_pool(v, ids.reshape(N, C * self.chunk_len), self.chunk_len)

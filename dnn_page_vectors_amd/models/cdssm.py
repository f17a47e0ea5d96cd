"""Convolutional DSSM (CDSSM) — reference parity model.

Tower (dssm_cnn_v2/cnn_dssm_th.py:83-139):
    Embedding(V, 100) -> Dropout(0.25) -> [Conv1D(150, k, valid, relu) -> MaxPool(L-k+1)]
    for k in (3, 4) -> concat (300) -> Dense(150) -> ReLU
One query tower and one document tower; the document tower is shared by the positive
and all J negatives (:147-156).  ``share_doc_tower=False`` gives the v1 layout with
independent towers per document slot (dssm_cnn/cnn_dssm.py:160-168) and
``final_dropout`` the v1 Dropout(0.5) before the last ReLU (:149).

Initialisation follows Keras 1 defaults: Embedding ``uniform`` U(-0.05, 0.05),
Convolution1D / Dense ``glorot_uniform`` (conv fans = input_dim*k, nb_filter*k),
zero biases.  Pretrained word vectors can be loaded into the embedding (word mode,
io/vectors.py).

Hot path: ``ops.conv_pool`` (fused gather/dropout/conv/max-pool, HIP) ->
``ops.dense.linear_act`` (fused bias+ReLU, HIP).
"""
from __future__ import annotations

import math
from typing import Dict, List

import torch
import torch.nn as nn

from ..ops import conv_pool as cops
from ..ops import dense as dops
from ..ops import reference as ref
from .base import TwoTowerModel


def glorot_uniform_(t: torch.Tensor, fan_in: int, fan_out: int, gen: torch.Generator) -> None:
    lim = math.sqrt(6.0 / (fan_in + fan_out))
    with torch.no_grad():
        t.uniform_(-lim, lim, generator=gen)


class CDSSMTower(nn.Module):
    def __init__(self, vocab_size: int, cfg, gen: torch.Generator):
        super().__init__()
        E, F = cfg.embedding_dim, cfg.num_filters
        self.widths = tuple(cfg.filter_sizes)
        self.embedding = nn.Parameter(torch.empty(vocab_size, E))
        with torch.no_grad():
            self.embedding.uniform_(-0.05, 0.05, generator=gen)
        self.conv_w = nn.ParameterList()
        self.conv_b = nn.ParameterList()
        for k in self.widths:
            w = nn.Parameter(torch.empty(F, k, E))
            glorot_uniform_(w, E * k, F * k, gen)
            self.conv_w.append(w)
            self.conv_b.append(nn.Parameter(torch.zeros(F)))
        self.dense_w = nn.Parameter(torch.empty(cfg.hidden_dims, F * len(self.widths)))
        glorot_uniform_(self.dense_w, F * len(self.widths), cfg.hidden_dims, gen)
        self.dense_b = nn.Parameter(torch.zeros(cfg.hidden_dims))
        self.p = float(cfg.dropout_prob[0])
        self.p_final = float(cfg.dropout_prob[1]) if cfg.final_dropout else 0.0
        self.mode = cfg.embed_dropout_mode
        self.act = getattr(cfg, "cdssm_act", "relu")  # Dense activation (reference: ReLU, cnn_dssm_th.py:136-138)

    def fast_ok(self) -> bool:
        return cops.fast_path_supported(self.embedding.shape[1], self.widths, self.conv_w[0].shape[0])

    def build_cache_ok(self) -> bool:
        return self.embedding.is_cuda and self.fast_ok() and cops.use_hip(self.embedding)

    def build_cache(self):
        if self.build_cache_ok():
            return (cops.table_bf16(self.embedding.detach()),
                    cops.pack_weights(self.conv_w[0].detach(), self.conv_w[1].detach()))
        return None

    def features(self, ids: torch.Tensor, training: bool, seed: int, cache=None) -> torch.Tensor:
        """The max-pooled, ReLU'd conv features (N, 2F) — cnn_dssm_th.py:86-134 before the Dense."""
        if ids.dtype != torch.int32:
            ids = ids.to(torch.int32)
        pooled, _ = cops.conv_relu_maxpool_fused(ids, self.embedding, list(self.conv_w), list(self.conv_b), self.p,
                                                 seed, training, self.mode, compute_cache=cache)
        return pooled

    def forward(self, ids: torch.Tensor, training: bool, seed: int, cache=None) -> torch.Tensor:
        return self.head(self.features(ids, training, seed, cache), training)

    def head(self, pooled: torch.Tensor, training: bool) -> torch.Tensor:
        """Dense + ReLU (cnn_dssm_th.py:136-138), with the v1 final dropout when configured."""
        if self.p_final > 0.0 and training:
            y = dops.linear_act(pooled, self.dense_w, self.dense_b, "none")
            y = torch.nn.functional.dropout(y, self.p_final, True)
            return torch.relu(y)
        return dops.linear_act(pooled, self.dense_w, self.dense_b, self.act)


class CDSSM(TwoTowerModel):
    def __init__(self, cfg, vocab_size: int):
        super().__init__(cfg)
        gen = torch.Generator().manual_seed(int(cfg.seed))
        self.vocab_size = vocab_size
        self.query_tower = CDSSMTower(vocab_size, cfg, gen)
        n_doc = 1 if cfg.share_doc_tower else 1 + cfg.J
        self.doc_towers = nn.ModuleList([CDSSMTower(vocab_size, cfg, gen) for _ in range(n_doc)])

    @property
    def out_dim(self) -> int:
        return self.cfg.hidden_dims

    def build_cache(self) -> Dict[str, object]:
        towers = [("query", self.query_tower)] + [(f"doc{i}", t) for i, t in enumerate(self.doc_towers)]
        if cops.PREP_MULTI and all(t.build_cache_ok() for _, t in towers):  # every tower's copies in one launch
            res = cops.prep_towers([(t.embedding.detach(), t.conv_w[0].detach(), t.conv_w[1].detach())
                                    for _, t in towers])
            return {k: r for (k, _), r in zip(towers, res)}
        c = {"query": self.query_tower.build_cache()}
        for i, t in enumerate(self.doc_towers):
            c[f"doc{i}"] = t.build_cache()
        return c

    def tower_forward(self, tower: str, ids: torch.Tensor, training: bool, seed: int, slot: int = 0) -> torch.Tensor:
        cache = self.compute_cache()
        if tower == "query":
            return self.query_tower(ids, training, seed, cache.get("query"))
        i = slot if len(self.doc_towers) > 1 else 0
        return self.doc_towers[i](ids, training, seed, cache.get(f"doc{i}"))


def cdssm_flops_per_sample(cfg) -> float:
    """Forward FLOPs of one (query + (1+J) docs) sample (2*MAC, conv + dense)."""
    E, F = cfg.embedding_dim, cfg.num_filters

    def tower(L):
        conv = sum(2 * (L - k + 1) * k * E * F for k in cfg.filter_sizes)
        return conv + 2 * F * len(cfg.filter_sizes) * cfg.hidden_dims

    return tower(cfg.query_length) + (1 + cfg.J) * tower(cfg.document_length)

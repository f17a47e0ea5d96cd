"""Two-tower MLP DSSM (BASELINE configs 1 and 3).

The classic DSSM architecture the reference's equations (4)/(5) come from
(dssm_cnn_v2/cnn_dssm_th.py:159-176 cite "equation (4)/(5)"): a letter-trigram
bag-of-words (hashed trigram ids, id 0 = pad) -> dense stack -> semantic vector,
scored by cosine with the gamma-softmax head.  ``mlp_dims = (d1, ..., dk)``:

    h1 = act(mean_t W1[ids_t] + b1)          (d1)   # multi-hot x W1 == embedding bag
    h_i = act(h_{i-1} W_i^T + b_i)           (d_i)
    out = h_{k-1} W_k^T + b_k                (d_k)  # linear semantic layer

Config 1: (300, 300, 128) over 1k hashed trigrams, batch 32 on CPU.
Config 3: (512, 512, 128) over 30k hashed trigrams with cross-GPU in-batch negatives.
Hot path: ``ops.embedding.embedding_bag`` (HIP gather for short bags, counts-matrix
GEMM for long pages) + ``ops.dense.linear_act`` (HIP MFMA, fused bias + tanh/ReLU).
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn

from ..ops import dense as dops
from ..ops import embedding as eops
from ..ops import fp8 as fops
from ..ops.optim import mirror_for
from .base import TwoTowerModel
from .cdssm import glorot_uniform_


class MLPTower(nn.Module):
    def __init__(self, vocab_size: int, dims, act: str, gen: torch.Generator, use_fp8: bool = False):
        super().__init__()
        self.use_fp8 = use_fp8
        # set by the owner for towers that see long bags (the chunked encoder's doc tower): with
        # use_fp8 their bag runs the counts plan on the block-scaled fp8 MFMA (ops/embedding.py)
        self.long_bags = False
        d1 = dims[0]
        self.embedding = nn.Parameter(torch.empty(vocab_size, d1))
        lim = math.sqrt(6.0 / (vocab_size + d1)) * math.sqrt(vocab_size / 64.0)  # bag mean of ~64 tokens
        with torch.no_grad():
            self.embedding.uniform_(-min(lim, 0.5), min(lim, 0.5), generator=gen)
            self.embedding[0].zero_()
        self.b1 = nn.Parameter(torch.zeros(d1))
        self.ws = nn.ParameterList()
        self.bs = nn.ParameterList()
        for a, b in zip(dims[:-1], dims[1:]):
            w = nn.Parameter(torch.empty(b, a))
            glorot_uniform_(w, a, b, gen)
            self.ws.append(w)
            self.bs.append(nn.Parameter(torch.zeros(b)))
        self.act = act

    def build_cache(self):
        m = mirror_for(self.embedding)  # written by the optimizer kernel with the last update
        c = {"emb16": m if m is not None else self.embedding.detach().to(torch.bfloat16).contiguous()}
        if self.use_fp8:
            c["w8"] = [fops.quantize(w.detach()) for w in self.ws]
            if self.long_bags:
                V = self.embedding.shape[0]
                c["emb8"] = fops.quantize_t(self.embedding, -(-V // fops.MX_BK) * fops.MX_BK)
        return c

    def forward(self, ids: torch.Tensor, cache=None) -> torch.Tensor:
        if ids.dtype != torch.int32:
            ids = ids.to(torch.int32)
        cache = cache or {}
        if self.act in ("none", "relu", "tanh"):  # first bias + activation fused into the bag kernel
            h = eops.embedding_bag(ids, self.embedding, cache.get("emb16"), pad=0, mean=True, bias=self.b1,
                                   act=self.act, fp8=self.use_fp8, w8=cache.get("emb8"))
            return self.dense_stack(h, cache, first_done=True)
        h = eops.embedding_bag(ids, self.embedding, cache.get("emb16"), pad=0, mean=True, fp8=self.use_fp8,
                               w8=cache.get("emb8"))
        return self.dense_stack(h, cache)

    def dense_stack(self, h: torch.Tensor, cache=None, first_done: bool = False) -> torch.Tensor:
        cache = cache or {}
        if not first_done:
            h = _bias_act(h, self.b1, self.act)
        n = len(self.ws)
        w8 = cache.get("w8")
        for i, (w, b) in enumerate(zip(self.ws, self.bs)):
            a = self.act if i < n - 1 else "none"
            if self.use_fp8:
                h = fops.fp8_linear(h, w, b, a, w8[i] if w8 is not None else None)
            else:
                h = dops.linear_act(h, w, b, a)
        return h


def mlp_tower_flops(L: int, dims) -> float:
    """Forward model FLOPs of one MLP tower over an L-token bag: the bag mean (L x d1 adds) +
    2 x MAC of the dense stack (bias / activation not counted, as for the CDSSM count)."""
    return float(L * dims[0] + sum(2 * a * b for a, b in zip(dims[:-1], dims[1:])))


def mlp_bag_gemm_flops(V: int, d1: int) -> float:
    """MFMA FLOPs the counts-matrix bag plan EXECUTES per long bag (2 x V x d1: the dense
    counts row times the table), for hardware-utilisation figures; most of it multiplies zeros."""
    return 2.0 * V * d1


def _bias_act(h: torch.Tensor, b: torch.Tensor, act: str) -> torch.Tensor:
    h = h + b
    if act == "tanh":
        return torch.tanh(h)
    if act == "relu":
        return torch.relu(h)
    return h


class MLPDSSM(TwoTowerModel):
    def __init__(self, cfg, vocab_size: int):
        super().__init__(cfg)
        gen = torch.Generator().manual_seed(int(cfg.seed))
        act = getattr(cfg, "mlp_act", "tanh")
        self.vocab_size = vocab_size
        self.query_tower = MLPTower(vocab_size, cfg.mlp_dims, act, gen)
        self.doc_towers = nn.ModuleList([MLPTower(vocab_size, cfg.mlp_dims, act, gen)])

    @property
    def out_dim(self) -> int:
        return self.cfg.mlp_dims[-1]

    def bf16_mirror_params(self):
        return [n for n, _ in self.named_parameters() if n.endswith(".embedding")]

    def build_cache(self):
        c = {}
        if self.query_tower.embedding.is_cuda:
            c["query"] = self.query_tower.build_cache()
            c["doc0"] = self.doc_towers[0].build_cache()
        return c

    def tower_forward(self, tower: str, ids: torch.Tensor, training: bool, seed: int, slot: int = 0) -> torch.Tensor:
        cache = self.compute_cache()
        if tower == "query":
            return self.query_tower(ids, cache.get("query"))
        return self.doc_towers[0](ids, cache.get("doc0"))

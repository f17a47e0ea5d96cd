"""BERT-base dual encoder (BASELINE config 4: "BERT-base dual-encoder page embedding,
DP=8 RCCL all-reduce over xGMI").

The reference only has the two-tower pattern (dssm_cnn_v2/cnn_dssm_th.py:147-176); this
model plugs a 12-layer / 768-hidden / 12-head Transformer encoder into it (shared
weights for queries and pages by default, ``[CLS]`` pooling, optional projection),
trained with the same cosine softmax head (in-batch / cross-GPU negatives).

MI355X mapping: every projection is a bf16 GEMM (hipBLASLt) over a cached bf16 copy of
the fp32 master weight (refreshed once per optimizer step; fp32 weight gradients);
attention is one fused HIP kernel pair on the packed QKV layout (csrc/kernels/
attention.hip: online softmax, no S/P materialisation, no head permutes); residual-add
+ LayerNorm and bias + GELU are fused HIP row kernels (transformer.hip); master weights
are fp32 in the flat parameter buffer (one bucketed all-reduce stream, ~440 MB/step at
BERT-base, overlapped with the backward by parallel/ddp.py).
Token ids come from the hashed word featurizer (no WordPiece vocab is available
offline); id 0 = [PAD], position 0 of every sequence is treated as [CLS].
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..ops import grad_sink
from ..ops import transformer as tops
from ..parallel.sparse_rows import note_rows
from .base import TwoTowerModel


class BertLayer(nn.Module):
    def __init__(self, H: int, I: int, heads: int):
        super().__init__()
        self.heads = heads
        self.wqkv = nn.Parameter(torch.empty(3 * H, H))
        self.bqkv = nn.Parameter(torch.zeros(3 * H))
        self.wo = nn.Parameter(torch.empty(H, H))
        self.bo = nn.Parameter(torch.zeros(H))
        self.ln1_g = nn.Parameter(torch.ones(H))
        self.ln1_b = nn.Parameter(torch.zeros(H))
        self.w1 = nn.Parameter(torch.empty(I, H))
        self.b1 = nn.Parameter(torch.zeros(I))
        self.w2 = nn.Parameter(torch.empty(H, I))
        self.b2 = nn.Parameter(torch.zeros(H))
        self.ln2_g = nn.Parameter(torch.ones(H))
        self.ln2_b = nn.Parameter(torch.zeros(H))

    def forward(self, x: torch.Tensor, mask: torch.Tensor, dt: torch.dtype, p_drop: float, training: bool,
                seed: int = 0):
        N, L, H = x.shape
        p = p_drop if training else 0.0
        r1, r2, bl = tops.ResidualLink(), tops.ResidualLink(), tops.BiasGradLink()
        qkv = tops.linear(x, self.wqkv, self.bqkv, res=r1, bias_link=bl)  # (N, L, 3H) [slot][head][d]
        a = tops.fused_attention(qkv, mask, self.heads, bias_link=bl)     # (N, L, H), no permute copies
        o = tops.linear(a, self.wo)
        # output bias + hidden dropout fused into the residual add + LayerNorm (counter-hash
        # masks; the bias gradient is reduced in the LayerNorm backward)
        x = tops.add_layernorm(o, x, self.ln1_g, self.ln1_b, p=p, seed=seed, bias=self.bo, res=r1)
        f2 = tops.ffn(x, self.w1, self.b1, self.w2, res=r2)  # GELU in the GEMM epilogues
        return tops.add_layernorm(f2, x, self.ln2_g, self.ln2_b, p=p, seed=(seed + 0x5BD1E995) & 0xFFFFFFFF,
                                  bias=self.b2, res=r2)


    def forward_packed(self, x: torch.Tensor, masks, shapes, p_drop: float, training: bool, seed: int = 0):
        """x (T, H): several sequence groups packed token-major (see BertEncoder.forward_multi)."""
        p = p_drop if training else 0.0
        # each x feeds a linear layer and a residual add: their gradients meet in the
        # linear's dX GEMM (tops.ResidualLink) instead of an autograd add
        r1, r2, bl = tops.ResidualLink(), tops.ResidualLink(), tops.BiasGradLink()
        qkv = tops.linear(x, self.wqkv, self.bqkv, res=r1, bias_link=bl)  # (T, 3H): one GEMM, all groups
        a = tops.packed_attention(qkv, masks, shapes, self.heads, bias_link=bl)
        o = tops.linear(a, self.wo)
        x = tops.add_layernorm(o, x, self.ln1_g, self.ln1_b, p=p, seed=seed, bias=self.bo, res=r1)
        f2 = tops.ffn(x, self.w1, self.b1, self.w2, res=r2)  # GELU in the GEMM epilogues
        return tops.add_layernorm(f2, x, self.ln2_g, self.ln2_b, p=p, seed=(seed + 0x5BD1E995) & 0xFFFFFFFF,
                                  bias=self.b2, res=r2)


def _row_gather(ids, W):
    note_rows(W, ids)  # sparse-gradient tables (parallel/sparse_rows.py) record their rows
    return _RowGather.apply(ids, W)


class _RowGather(torch.autograd.Function):
    """Token-embedding lookup whose backward is an atomic row scatter (``index_add_``).

    ``F.embedding``'s backward sorts the ids and runs a rocPRIM ``unique_by_key``; replayed
    inside a hipGraph that kernel hit a memory-aperture fault on MI355X / ROCm 7.2 (BERT
    bench, graph mode).  The scatter form has no library scan in it, and at BERT's
    270k tokens x 768 per step it is a few hundred microseconds either way.
    """

    @staticmethod
    def forward(ctx, ids, W):
        flat = ids.reshape(-1)
        ctx.save_for_backward(flat)
        ctx.shape = W.shape
        ctx.W = W  # flat-gradient direct-write target (ops/grad_sink.py)
        return W.index_select(0, flat).view(*ids.shape, W.shape[1])

    @staticmethod
    def backward(ctx, g):
        (flat,) = ctx.saved_tensors
        gf = g.reshape(-1, ctx.shape[1]).float()
        tw = grad_sink.accum_target(ctx.W)  # the scatter accumulates: add straight into the flat grad
        if tw is not None:
            tw.index_add_(0, flat, gf)
            grad_sink.done(ctx.W)
            return None, None
        gW = torch.zeros(ctx.shape, dtype=torch.float32, device=g.device)
        gW.index_add_(0, flat, gf)
        return None, gW


class BertEncoder(nn.Module):
    def __init__(self, vocab_size: int, H: int, I: int, heads: int, layers: int, max_len: int, out_dim: int,
                 gen: torch.Generator):
        super().__init__()
        self.word = nn.Parameter(torch.empty(vocab_size, H))
        self.pos = nn.Parameter(torch.empty(max_len, H))
        self.typ = nn.Parameter(torch.empty(2, H))
        self.ln_g = nn.Parameter(torch.ones(H))
        self.ln_b = nn.Parameter(torch.zeros(H))
        self.layers = nn.ModuleList([BertLayer(H, I, heads) for _ in range(layers)])
        self.proj = nn.Parameter(torch.empty(out_dim, H)) if out_dim else None
        with torch.no_grad():
            for n, p in self.named_parameters():
                if p.dim() == 2:
                    p.normal_(0.0, 0.02, generator=gen)

    def forward(self, ids: torch.Tensor, p_drop: float, training: bool, seed: int = 0) -> torch.Tensor:
        dt = torch.bfloat16 if ids.is_cuda else torch.float32
        ids = ids.long()
        N, L = ids.shape
        mask = (ids != 0)
        mask[:, 0] = True  # [CLS] position always attends
        x = (_row_gather(ids, self.word) + self.pos[:L].unsqueeze(0) + self.typ[0]).to(dt)
        x = tops.add_layernorm(x, None, self.ln_g, self.ln_b)
        if training and p_drop > 0:
            x = F.dropout(x, p_drop, True)
        for li, layer in enumerate(self.layers):
            x = layer(x, mask, dt, p_drop, training, seed=(int(seed) * 1000003 + li * 7919) & 0xFFFFFFFF)
        cls = x[:, 0].float()
        return F.linear(cls, self.proj) if self.proj is not None else cls

    def forward_multi(self, ids_list, p_drop: float, training: bool, seed: int = 0):
        """Several id batches (e.g. the queries (B, Lq) and the pages (B*S, Ld) of one step)
        through the SAME encoder in one pass: every position-wise op (the four linear layers,
        bias+GELU, residual+LayerNorm, their backward and weight gradients) runs once over the
        packed tokens; only attention is per group.  Each weight then receives one gradient
        (no accumulation adds) from one larger, better-filled GEMM.  Returns the per-group
        CLS vectors (projected if configured)."""
        dt = torch.bfloat16 if ids_list[0].is_cuda else torch.float32
        xs, masks, shapes = [], [], []
        for ids in ids_list:
            N, L = ids.shape
            mask = (ids != 0).to(torch.int32)  # int32 once: the attention kernels' layout (no per-layer cast)
            mask[:, 0] = 1
            masks.append(mask)
            shapes.append((N, L))
        # one fused gather + position / type add + cast over every group (ops/transformer.py)
        x = tops.bert_embed(self.word, self.pos, self.typ, ids_list)
        if x is None:
            for ids in ids_list:
                ids = ids.long()
                N, L = ids.shape
                xs.append((_row_gather(ids, self.word) + self.pos[:L].unsqueeze(0) + self.typ[0]).to(dt)
                          .reshape(N * L, -1))
            x = torch.cat(xs, 0) if len(xs) > 1 else xs[0]
        x = tops.add_layernorm(x, None, self.ln_g, self.ln_b)
        if training and p_drop > 0:
            x = F.dropout(x, p_drop, True)
        for li, layer in enumerate(self.layers):
            x = layer.forward_packed(x, masks, shapes, p_drop, training,
                                     seed=(int(seed) * 1000003 + li * 7919) & 0xFFFFFFFF)
        outs, off = [], 0
        for N, L in shapes:
            cls = x[off:off + N * L].view(N, L, -1)[:, 0].float()
            off += N * L
            outs.append(F.linear(cls, self.proj) if self.proj is not None else cls)
        return outs


class BertDualEncoder(TwoTowerModel):
    def __init__(self, cfg, vocab_size: int):
        super().__init__(cfg)
        gen = torch.Generator().manual_seed(int(cfg.seed))
        self.vocab_size = vocab_size
        mk = lambda: BertEncoder(vocab_size, cfg.bert_hidden, cfg.bert_intermediate, cfg.bert_heads,
                                 cfg.bert_layers, cfg.bert_max_len, cfg.bert_out_dim, gen)
        self.query_tower = mk()
        # siamese by default: the page tower IS the query tower (one set of weights)
        self.doc_towers = nn.ModuleList([self.query_tower] if cfg.share_doc_tower else [mk()])
        self.p_drop = float(getattr(cfg, "bert_dropout", 0.1))

    @property
    def out_dim(self) -> int:
        return self.cfg.bert_out_dim or self.cfg.bert_hidden

    def bf16_mirror_params(self):
        return [n for n, _ in self.named_parameters() if n.rsplit(".", 1)[-1] in ("wqkv", "wo", "w1", "w2")]

    def tower_forward(self, tower: str, ids: torch.Tensor, training: bool, seed: int, slot: int = 0) -> torch.Tensor:
        enc = self.query_tower if tower == "query" else self.doc_towers[0]
        return enc(ids, self.p_drop, training, seed=seed)

    def forward(self, q_ids: torch.Tensor, d_ids: torch.Tensor, seed: int = 0, doc_hook=None):
        """Siamese towers: queries and pages of the step go through the encoder as ONE packed
        token batch (BertEncoder.forward_multi); separate towers use the base class path."""
        if self.doc_towers[0] is not self.query_tower or not getattr(self.cfg, "bert_packed", True):
            return super().forward(q_ids, d_ids, seed=seed, doc_hook=doc_hook)
        B, S, Ld = d_ids.shape
        qv, dv = self.query_tower.forward_multi([q_ids, d_ids.reshape(B * S, Ld)], self.p_drop, self.training,
                                                seed=seed * 2 + 1)
        d = dv.view(B, S, -1)
        if doc_hook is not None:
            doc_hook(d)
        return qv, d


def bert_flops_per_token(cfg, L: int) -> float:
    H, I, Lyr = cfg.bert_hidden, cfg.bert_intermediate, cfg.bert_layers
    return Lyr * (2 * (4 * H * H + 2 * H * I) + 4 * L * H)

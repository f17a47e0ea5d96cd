"""Transformer ops for the BERT dual encoder: fused residual-add + LayerNorm, fused
bias + GELU, masked softmax attention (HIP row kernels around hipBLASLt GEMMs).

CPU: plain torch (the reference semantics).  GPU activations are bf16; LayerNorm
statistics and parameter gradients are fp32.
"""
from __future__ import annotations

import math
from typing import Optional

import torch
import torch.nn.functional as F

from ._common import P, check, lib, stream, use_hip


class _AddLNFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, r, gamma, beta, eps):
        x = x.to(torch.bfloat16).contiguous()
        r = r.to(torch.bfloat16).contiguous() if r is not None else None
        D = x.shape[-1]
        M = x.numel() // D
        y = torch.empty_like(x)
        h = torch.empty_like(x)
        mean = torch.empty(M, dtype=torch.float32, device=x.device)
        rstd = torch.empty(M, dtype=torch.float32, device=x.device)
        check(lib().pv_add_layernorm_fwd(P(x), P(r), P(gamma), P(beta), P(y), P(h), P(mean), P(rstd), M, D, eps,
                                         stream(x.device)), "pv_add_layernorm_fwd")
        ctx.save_for_backward(h, gamma, mean, rstd)
        ctx.has_r = r is not None
        return y

    @staticmethod
    def backward(ctx, dy):
        h, gamma, mean, rstd = ctx.saved_tensors
        D = h.shape[-1]
        M = h.numel() // D
        dy = dy.to(torch.bfloat16).contiguous()
        dx = torch.empty_like(h)
        dg = torch.zeros_like(gamma)
        db = torch.zeros_like(gamma)
        check(lib().pv_layernorm_bwd(P(dy), P(h), P(gamma), P(mean), P(rstd), P(dx), P(dg), P(db), M, D,
                                     stream(h.device)), "pv_layernorm_bwd")
        return dx, (dx if ctx.has_r else None), dg, db, None


def add_layernorm(x: torch.Tensor, r: Optional[torch.Tensor], gamma: torch.Tensor, beta: torch.Tensor,
                  eps: float = 1e-12) -> torch.Tensor:
    if use_hip(x):
        return _AddLNFn.apply(x, r, gamma, beta, eps)
    h = x if r is None else x + r
    return F.layer_norm(h.float(), (h.shape[-1],), gamma, beta, eps).to(x.dtype)


class _BiasGeluFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, b):
        x = x.to(torch.bfloat16).contiguous()
        y = torch.empty_like(x)
        D = x.shape[-1]
        check(lib().pv_bias_gelu_fwd(P(x), P(b), P(y), x.numel(), D, stream(x.device)), "pv_bias_gelu_fwd")
        ctx.save_for_backward(x, b)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, b = ctx.saved_tensors
        D = x.shape[-1]
        M = x.numel() // D
        dy = dy.to(torch.bfloat16).contiguous()
        dx = torch.empty_like(x)
        db = torch.zeros_like(b)
        L_ = lib()
        ws = torch.empty(L_.pv_bias_gelu_bwd_ws(M, D), dtype=torch.float32, device=x.device) if D % 8 == 0 else None
        check(L_.pv_bias_gelu_bwd(P(x), P(b), P(dy), P(dx), P(db), P(ws), M, D, stream(x.device)), "pv_bias_gelu_bwd")
        return dx, db


def bias_gelu(x: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    if use_hip(x):
        return _BiasGeluFn.apply(x, b)
    return F.gelu(x + b, approximate="tanh")


class _SoftmaxFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, s, mask, scale, heads):
        s = s.to(torch.bfloat16).contiguous()
        L = s.shape[-1]
        R = s.numel() // L
        rows_per_item = heads * s.shape[-2]
        check(lib().pv_softmax_fwd(P(s), P(mask), R, L, rows_per_item, scale, stream(s.device)), "pv_softmax_fwd")
        ctx.save_for_backward(s)
        ctx.scale = scale
        return s

    @staticmethod
    def backward(ctx, dp):
        p, = ctx.saved_tensors
        L = p.shape[-1]
        R = p.numel() // L
        d = dp.to(torch.bfloat16).contiguous().clone()
        check(lib().pv_softmax_bwd(P(p), P(d), R, L, ctx.scale, stream(p.device)), "pv_softmax_bwd")
        return d, None, None, None


def attention(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, mask: Optional[torch.Tensor]) -> torch.Tensor:
    """q, k, v: (B, H, L, d); mask (B, L) int (1 = real token). Returns (B, H, L, d)."""
    scale = 1.0 / math.sqrt(q.shape[-1])
    if use_hip(q):
        s = torch.matmul(q, k.transpose(-1, -2))                 # hipBLASLt, bf16
        m = mask.to(torch.int32).contiguous() if mask is not None else None
        p = _SoftmaxFn.apply(s, m, scale, q.shape[1])
        return torch.matmul(p, v)
    s = torch.matmul(q.float(), k.float().transpose(-1, -2)) * scale
    if mask is not None:
        s = s.masked_fill(~mask.bool()[:, None, None, :], float("-inf"))
    return torch.matmul(torch.softmax(s, -1), v.float()).to(q.dtype)

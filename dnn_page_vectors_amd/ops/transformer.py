"""Transformer ops for the BERT dual encoder: fused residual-add + LayerNorm, fused
bias + GELU, fused multi-head attention on the packed QKV layout, and a bf16 linear layer
over cached bf16 weights (HIP kernels around hipBLASLt GEMMs).

CPU: plain torch (the reference semantics).  GPU activations are bf16; LayerNorm
statistics and parameter gradients are fp32.
"""
from __future__ import annotations

import math
import os
from typing import Optional

import torch
import torch.nn.functional as F

from . import dense as dops
from . import grad_sink
from . import reference as ref
from ._common import P, check, lib, stream, use_hip


def _seed_ptr():
    """Device seed offset of a captured hipGraph step (ops.conv_pool.set_seed_tensor): the
    fused dropout kernels add it so each replay draws fresh masks."""
    from . import conv_pool

    return conv_pool._SEED_DEV


RESID_FUSE = os.environ.get("PAGEVEC_RESID_FUSE", "1") != "0"


class ResidualLink:
    """Pairs a residual add (``add_layernorm(..., r=x, res=link)``) with the linear layer
    that reads the same x (``linear(x, ..., res=link)``).  Autograd would sum the two
    gradients of x with a separate bf16 add over (tokens x hidden) per residual (1.3 ms
    of a BERT-base step); instead the LayerNorm backward parks its residual gradient here
    and the linear layer's backward adds it in the dX GEMM's epilogue (addmm, beta = 1).
    The LayerNorm backward always runs first: the linear's output gradient depends on it."""

    __slots__ = ("grad",)

    def __init__(self):
        self.grad = None


class BiasGradLink:
    """Pairs the qkv projection (``linear(x, w, b, bias_link=link)``) with the attention that
    consumes its output (``packed_attention(..., bias_link=link)``).  The qkv bias gradient is
    the column sum of dqkv over every token (T x 3H bf16, re-read from HBM by a colsum pass); the
    attention backward kernels already hold dQ / dK / dV in registers and emit per-workgroup
    column sums instead (attention.hip::pv_attn_bwd2, ``part``: (sum N_i ceil(L_i / 64), 3H)
    fp32, ~50x fewer rows), which the linear's backward reduces into the bias gradient.  The
    attention backward always runs first: the linear's output gradient is its dqkv."""

    __slots__ = ("part",)

    def __init__(self):
        self.part = None


# qkv bias gradient from the attention backward's partial column sums (BiasGradLink)
ATTN_BGRAD = os.environ.get("PAGEVEC_ATTN_BGRAD", "1") != "0"


class _AddLNFn(torch.autograd.Function):
    """y = LayerNorm(dropout(x + xb) + r).  D in {256, 512, 768, 1024}: one wave per row
    (``pv_add_ln_drop_fwd``); the dropout mask is a counter hash of (seed, row, column)
    (ops/reference.py::dropout_keep_mask, p quantised to 1/256), regenerated in the backward,
    which writes both the residual gradient and the masked branch gradient in one pass and
    reduces the branch bias gradient (column sums) with the LayerNorm parameter gradients.
    ``xb``: the bias of the linear layer producing x (that GEMM then runs without one)."""

    @staticmethod
    def forward(ctx, x, r, gamma, beta, eps, p, seed, xb, res=None):
        x = x.to(torch.bfloat16).contiguous()
        r = r.to(torch.bfloat16).contiguous() if r is not None else None
        D = x.shape[-1]
        M = x.numel() // D
        y = torch.empty_like(x)
        h = torch.empty_like(x)
        mean = torch.empty(M, dtype=torch.float32, device=x.device)
        rstd = torch.empty(M, dtype=torch.float32, device=x.device)
        thr = ref.dropout_threshold(p) if p > 0 else 0
        scale = 256.0 / (256.0 - thr)
        sp = _seed_ptr() if thr > 0 else None
        seed = int(seed) & 0xFFFFFFFF
        xbf = xb.float().contiguous() if xb is not None else None
        if D in _LN_ROWS:
            check(lib().pv_add_ln_drop_fwd(P(x), P(xbf), P(r), P(gamma), P(beta), P(y), P(h), P(mean), P(rstd), M, D,
                                           eps, thr, scale, seed, P(sp), stream(x.device)), "pv_add_ln_drop_fwd")
        else:
            if thr > 0 or xb is not None:
                raise ValueError(f"fused dropout / bias + LayerNorm needs D in {_LN_ROWS}")
            check(lib().pv_add_layernorm_fwd(P(x), P(r), P(gamma), P(beta), P(y), P(h), P(mean), P(rstd), M, D, eps,
                                             stream(x.device)), "pv_add_layernorm_fwd")
        ctx.save_for_backward(h, gamma, mean, rstd, sp)
        ctx.has_r = r is not None
        ctx.drop = (thr, scale, seed)
        ctx.xb = None if xb is None else (xb.shape, xb.dtype)
        ctx.params = (gamma, beta, xb)  # flat-gradient direct-write targets (ops/grad_sink.py)
        ctx.res = res if (r is not None and RESID_FUSE) else None
        return y

    @staticmethod
    def backward(ctx, dy):
        h, gamma, mean, rstd, sp = ctx.saved_tensors
        thr, scale, seed = ctx.drop
        D = h.shape[-1]
        M = h.numel() // D
        dy = dy.to(torch.bfloat16).contiguous()
        dx = torch.empty_like(h)
        L_ = lib()
        nws = int(L_.pv_layernorm_bwd_ws(M, D))
        alloc = torch.empty if nws > 0 else torch.zeros  # generic kernel accumulates atomically
        # the workspace path overwrites dg / db / dxb: write them straight into the flat
        # gradient when this is the parameters' first contribution (ops/grad_sink.py)
        tgt = [grad_sink.write_target(q) if (nws > 0 and ctx.needs_input_grad[i]) else None
               for q, i in zip(ctx.params, (2, 3, 7))]
        dg = tgt[0] if tgt[0] is not None else alloc(gamma.shape, dtype=torch.float32, device=h.device)
        db = tgt[1] if tgt[1] is not None else alloc(gamma.shape, dtype=torch.float32, device=h.device)
        ws = torch.empty(nws, dtype=torch.float32, device=h.device) if nws > 0 else None
        dxb = None
        if ctx.xb is not None:
            dxb = tgt[2] if tgt[2] is not None else torch.empty(D, dtype=torch.float32, device=h.device)
        if thr > 0 or dxb is not None:
            dxm = torch.empty_like(h) if thr > 0 else None
            check(L_.pv_layernorm_bwd_drop(P(dy), P(h), P(gamma), P(mean), P(rstd), P(dx), P(dxm), P(dg), P(db),
                                           P(dxb), P(ws), M, D, thr, scale, seed, P(sp), stream(h.device)),
                  "pv_layernorm_bwd_drop")
            if dxm is None:
                dxm = dx
        else:
            dxm = dx
            check(L_.pv_layernorm_bwd(P(dy), P(h), P(gamma), P(mean), P(rstd), P(dx), P(dg), P(db), P(ws), M, D,
                                      stream(h.device)), "pv_layernorm_bwd")
        if dxb is not None and ctx.xb[1] != torch.float32:
            dxb = dxb.to(ctx.xb[1])
        outs = [dg, db, dxb]
        for j, (t, q) in enumerate(zip(tgt, ctx.params)):
            if t is not None:
                grad_sink.done(q)
                outs[j] = None
        dr = dx if ctx.has_r else None
        if dr is not None and ctx.res is not None and ctx.needs_input_grad[1]:
            ctx.res.grad = dr  # the paired linear layer's dX GEMM adds it (ResidualLink)
            dr = None
        return dxm, dr, outs[0], outs[1], None, None, None, outs[2], None


_LN_ROWS = (256, 512, 768, 1024)


def add_layernorm(x: torch.Tensor, r: Optional[torch.Tensor], gamma: torch.Tensor, beta: torch.Tensor,
                  eps: float = 1e-12, p: float = 0.0, seed: int = 0,
                  bias: Optional[torch.Tensor] = None, res: Optional[ResidualLink] = None) -> torch.Tensor:
    """LayerNorm(dropout_p(x + bias) + r) (dropout only when p > 0: pass p = 0 outside
    training; ``bias`` = the bias of the linear layer that produced x, folded in here)."""
    if use_hip(x):
        if x.shape[-1] not in _LN_ROWS:
            if bias is not None:
                x = x + bias.to(x.dtype)
                bias = None
            if p > 0:
                x = F.dropout(x, p, True)
                p = 0.0
        return _AddLNFn.apply(x, r, gamma, beta, eps, float(p), int(seed), bias, res)
    if bias is not None:
        x = x + bias.to(x.dtype)
    if p > 0:
        keep = ref.dropout_keep_mask(seed, x.numel() // x.shape[-1], x.shape[-1], p, device=x.device)
        x = x * keep.view(x.shape).to(x.dtype) * (256.0 / (256.0 - ref.dropout_threshold(p)))
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
        ctx.params = (b,)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, b = ctx.saved_tensors
        D = x.shape[-1]
        M = x.numel() // D
        dy = dy.to(torch.bfloat16).contiguous()
        dx = torch.empty_like(x)
        tb = grad_sink.write_target(ctx.params[0]) if (D % 8 == 0 and b.dtype == torch.float32
                                                       and ctx.needs_input_grad[1]) else None
        if tb is not None:
            db = tb
        else:
            db = torch.empty_like(b) if D % 8 == 0 else torch.zeros_like(b)  # vector path overwrites db
        L_ = lib()
        ws = torch.empty(L_.pv_bias_gelu_bwd_ws(M, D), dtype=torch.float32, device=x.device) if D % 8 == 0 else None
        check(L_.pv_bias_gelu_bwd(P(x), P(b), P(dy), P(dx), P(db), P(ws), M, D, stream(x.device)), "pv_bias_gelu_bwd")
        if tb is not None:
            grad_sink.done(ctx.params[0])
            db = None
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


class _FusedAttnFn(torch.autograd.Function):
    """qkv (N, L, 3*H*64) bf16 packed [slot][head][d] -> (N, L, H*64); csrc/kernels/attention.hip."""

    @staticmethod
    def forward(ctx, qkv, mask, heads, scale, blink=None):
        qkv = qkv.to(torch.bfloat16).contiguous()
        N, L, C = qkv.shape
        H = heads
        if C != 3 * H * 64:
            raise ValueError("fused attention needs head dim 64")
        out = torch.empty(N, L, H * 64, dtype=torch.bfloat16, device=qkv.device)
        lse = torch.empty(N, H, L, dtype=torch.float32, device=qkv.device)
        check(lib().pv_attn_fwd(P(qkv), P(mask), P(out), P(lse), N, L, H, float(scale), stream(qkv.device)),
              "pv_attn_fwd")
        ctx.save_for_backward(qkv, mask, out, lse)
        ctx.meta = (H, float(scale))
        ctx.blink = blink
        return out

    @staticmethod
    def backward(ctx, dout):
        qkv, mask, out, lse = ctx.saved_tensors
        H, scale = ctx.meta
        N, L, _ = qkv.shape
        dout = dout.to(torch.bfloat16).contiguous()
        D = torch.empty(N, H, L, dtype=torch.float32, device=qkv.device)
        dqkv = torch.empty_like(qkv)
        part = None
        if ctx.blink is not None:
            part = torch.zeros(N * ((L + 63) // 64), 3 * H * 64, dtype=torch.float32, device=qkv.device)
            ctx.blink.part = part
        check(lib().pv_attn_bwd2(P(qkv), P(mask), P(out), P(dout), P(lse), P(D), P(dqkv), N, L, H, scale,
                                 P(part), stream(qkv.device)), "pv_attn_bwd2")
        return dqkv, None, None, None, None


def fused_attention(qkv: torch.Tensor, mask: Optional[torch.Tensor], heads: int,
                    bias_link: Optional[BiasGradLink] = None) -> torch.Tensor:
    """qkv (N, L, 3*H*d) packed projection output -> attention output (N, L, H*d), mask (N, L).
    ``bias_link``: shared with the qkv ``linear`` (BiasGradLink)."""
    N, L, C = qkv.shape
    d = C // (3 * heads)
    scale = 1.0 / math.sqrt(d)
    if use_hip(qkv) and d == 64:
        m = mask.to(torch.int32).contiguous() if mask is not None else None
        return _FusedAttnFn.apply(qkv, m, heads, scale, bias_link if ATTN_BGRAD else None)
    q, k, v = qkv.view(N, L, 3, heads, d).permute(2, 0, 3, 1, 4)
    return attention(q, k, v, mask).transpose(1, 2).reshape(N, L, heads * d)


class _PackedAttnFn(torch.autograd.Function):
    """Attention over several packed sequence groups in ONE token-major tensor: qkv (T, 3*H*64)
    holds segments of (N_i, L_i) sequences back to back (the query and the page tower of the
    siamese dual encoder); each segment runs the fused kernels on offset pointers into the
    shared input / output / gradient buffers — no per-tower copies, slices or gradient adds."""

    @staticmethod
    def forward(ctx, qkv, masks, shapes, heads, scale, blink=None):
        qkv = qkv.to(torch.bfloat16).contiguous()
        T, C = qkv.shape
        H = heads
        if C != 3 * H * 64:
            raise ValueError("fused attention needs head dim 64")
        out = torch.empty(T, H * 64, dtype=torch.bfloat16, device=qkv.device)
        lses = []
        off = 0
        s = stream(qkv.device)
        esz = qkv.element_size()
        for (N, L), m in zip(shapes, masks):
            lse = torch.empty(N, H, L, dtype=torch.float32, device=qkv.device)
            check(lib().pv_attn_fwd(qkv.data_ptr() + off * C * esz, P(m), out.data_ptr() + off * H * 64 * esz,
                                    P(lse), N, L, H, float(scale), s), "pv_attn_fwd")
            lses.append(lse)
            off += N * L
        if off != T:
            raise ValueError("segment shapes do not cover the packed tensor")
        ctx.save_for_backward(qkv, out, *masks, *lses)
        ctx.meta = (H, float(scale), list(shapes), len(masks))
        ctx.blink = blink
        return out

    @staticmethod
    def backward(ctx, dout):
        H, scale, shapes, k = ctx.meta
        saved = ctx.saved_tensors
        qkv, out, masks, lses = saved[0], saved[1], saved[2:2 + k], saved[2 + k:]
        T, C = qkv.shape
        dout = dout.to(torch.bfloat16).contiguous()
        dqkv = torch.empty_like(qkv)
        esz = qkv.element_size()
        s = stream(qkv.device)
        part, prow = None, 0
        if ctx.blink is not None:
            part = torch.zeros(sum(N * ((L + 63) // 64) for N, L in shapes), C, dtype=torch.float32,
                               device=qkv.device)
            ctx.blink.part = part
        off = 0
        for (N, L), m, lse in zip(shapes, masks, lses):
            D = torch.empty(N, H, L, dtype=torch.float32, device=qkv.device)
            check(lib().pv_attn_bwd2(qkv.data_ptr() + off * C * esz, P(m), out.data_ptr() + off * H * 64 * esz,
                                     dout.data_ptr() + off * H * 64 * esz, P(lse), P(D),
                                     dqkv.data_ptr() + off * C * esz, N, L, H, scale,
                                     part.data_ptr() + prow * C * 4 if part is not None else None, s),
                  "pv_attn_bwd2")
            off += N * L
            prow += N * ((L + 63) // 64)
        return dqkv, None, None, None, None, None


def packed_attention(qkv: torch.Tensor, masks, shapes, heads: int,
                     bias_link: Optional[BiasGradLink] = None) -> torch.Tensor:
    """qkv (T, 3*H*d) token-major with segments of shapes [(N_i, L_i)] back to back, masks
    [(N_i, L_i)] -> (T, H*d).  ``bias_link``: shared with the qkv ``linear`` (BiasGradLink)."""
    d = qkv.shape[1] // (3 * heads)
    if use_hip(qkv) and d == 64:
        ms = [m.to(torch.int32).contiguous() for m in masks]
        return _PackedAttnFn.apply(qkv, ms, [tuple(x) for x in shapes], heads, 1.0 / math.sqrt(d),
                                   bias_link if ATTN_BGRAD else None)
    outs, off = [], 0
    for (N, L), m in zip(shapes, masks):
        outs.append(fused_attention(qkv[off:off + N * L].view(N, L, -1), m, heads).reshape(N * L, -1))
        off += N * L
    return torch.cat(outs, 0)


class _BertEmbedFn(torch.autograd.Function):
    """BERT's embedding front end over the packed token batch: bf16(word[id] + pos[l] + typ[0])
    in one kernel (transformer.hip::bert_embed_fwd_kernel) instead of an fp32 gather, two
    broadcast adds, a cast and a cat per group.  Backward: the word-table rows by fp32 atomics
    straight from the bf16 gradient into the flat gradient (all-zero padding pieces skipped),
    the position rows as per-group sums over sequences, the type row as their total — each
    table receives ONE gradient (the per-group lookups of the old path made the word table a
    multi-use parameter: two zero-filled V x H temporaries, an add and a copy per step)."""

    @staticmethod
    def forward(ctx, word, pos, typ, ids_flat, groups):
        import ctypes

        T = ids_flat.numel()
        H = word.shape[1]
        out = torch.empty(T, H, dtype=torch.bfloat16, device=word.device)
        offs, lens = [], []
        off = 0
        for N, L in groups:
            offs.append(off)
            lens.append(L)
            off += N * L
        if off != T:
            raise ValueError("group shapes do not cover the packed ids")
        oa, la = (ctypes.c_int * 4)(*offs), (ctypes.c_int * 4)(*lens)
        check(lib().pv_bert_embed_fwd(P(ids_flat), P(word), P(pos), P(typ[0]), P(out), T, H,
                                      ctypes.cast(oa, ctypes.c_void_p), ctypes.cast(la, ctypes.c_void_p), len(groups),
                                      stream(word.device)), "pv_bert_embed_fwd")
        ctx.save_for_backward(ids_flat)
        ctx.groups = list(groups)
        ctx.params = (word, pos, typ)
        return out

    @staticmethod
    def backward(ctx, g):
        (ids_flat,) = ctx.saved_tensors
        word, pos, typ = ctx.params
        g = g.to(torch.bfloat16).contiguous()
        T, H = g.shape
        dword = dpos = dtyp = None
        if ctx.needs_input_grad[0]:
            tw = grad_sink.accum_target(word)
            dst = tw if tw is not None else torch.zeros(word.shape, dtype=torch.float32, device=g.device)
            check(lib().pv_bert_embed_wgrad(P(ids_flat), P(g), P(dst), T, H, stream(g.device)), "pv_bert_embed_wgrad")
            if tw is not None:
                grad_sink.done(word)
            else:
                dword = dst
        if ctx.needs_input_grad[1] or ctx.needs_input_grad[2]:
            dpos = torch.zeros(pos.shape, dtype=torch.float32, device=g.device)
            off = 0
            for N, L in ctx.groups:
                dpos[:L] += torch.sum(g[off:off + N * L].view(N, L, H), dim=0, dtype=torch.float32)
                off += N * L
            if ctx.needs_input_grad[2]:
                dtyp = torch.zeros(typ.shape, dtype=torch.float32, device=g.device)
                dtyp[0] = dpos.sum(0)
            if not ctx.needs_input_grad[1]:
                dpos = None
        return dword, dpos, dtyp, None, None


def bert_embed(word: torch.Tensor, pos: torch.Tensor, typ: torch.Tensor, ids_list) -> Optional[torch.Tensor]:
    """Packed (T, H) bf16 embeddings of several id batches, or None off the HIP path and in the
    deterministic mode (the word-table gradient here is float atomics; the per-group path's
    index_add_ is deterministic there)."""
    from . import determinism

    if not (use_hip(word) and word.shape[1] % 8 == 0 and len(ids_list) <= 4 and BERT_EMBED) \
            or determinism.enabled():
        return None
    from ..parallel.sparse_rows import note_rows

    flat = torch.cat([i.reshape(-1) for i in ids_list]).to(torch.int32) if len(ids_list) > 1 \
        else ids_list[0].reshape(-1).to(torch.int32)
    note_rows(word, flat)  # row-sparse table gradients (parallel/sparse_rows.py) record the rows
    return _BertEmbedFn.apply(word, pos, typ, flat.contiguous(), [tuple(i.shape) for i in ids_list])


BERT_EMBED = os.environ.get("PAGEVEC_BERT_EMBED", "1") != "0"


# bf16 copies of fp32 master weights, refreshed once per optimizer step (generation counter
# of models.base: bump_generation() after every update)
_W16 = {}


def weight_bf16(w: torch.Tensor) -> torch.Tensor:
    from ..models.base import _GENERATION
    from .optim import mirror_for

    m = mirror_for(w)  # the optimizer kernel's bf16 copy (FlatAdam(mirror=...))
    if m is not None:
        return m

    key = id(w)
    ent = _W16.get(key)
    if ent is None or ent[0] != _GENERATION[0] or ent[1] is not w or ent[2].shape != w.shape:
        ent = (_GENERATION[0], w, w.detach().to(torch.bfloat16))
        _W16[key] = ent
    return ent[2]


def _wgrad_splits(T: int) -> int:
    """Token-axis split count of the weight-gradient GEMM (a power of two dividing T)."""
    sk = 1
    while sk < 16 and T % (2 * sk) == 0 and T // (2 * sk) >= 2048:
        sk *= 2
    return sk


def wgrad_f32(dy2: torch.Tensor, x2: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """dW = dy^T x (bf16 operands, fp32 result) for T >> N, K.

    A single GEMM has only (N/256)(K/256) output tiles (36 for 768 x 3072) for a 65536-long
    reduction, so hipBLASLt runs it on a fraction of the 256 CUs (285-680 TF/s measured,
    tools/gemm_micro.py).  Splitting the token axis into up to 16 batched fp32-output GEMMs
    and summing the partials in fp32 fills the chip: 1.82 -> 1.03 ms per BERT layer at
    T = 65536 (bmm out_dtype=fp32; same fp32 accumulation, different summation order).
    ``out``: fp32 destination (a flat-gradient view, ops/grad_sink.py), overwritten.
    """
    T = dy2.shape[0]
    sk = _wgrad_splits(T)
    try:
        if sk == 1:
            return torch.mm(dy2.t(), x2, out_dtype=torch.float32, out=out)
        dy3 = dy2.view(sk, T // sk, dy2.shape[1])
        x3 = x2.view(sk, T // sk, x2.shape[1])
        return dops.colsum(torch.bmm(dy3.transpose(1, 2), x3, out_dtype=torch.float32), out=out)
    except (TypeError, RuntimeError, NotImplementedError):  # no mm/bmm out_dtype (CPU)
        r = dy2.t().float() @ x2.float()
        return r if out is None else out.copy_(r)


class _Linear16Fn(torch.autograd.Function):
    """y = x @ W^T (+ b) in bf16 on hipBLASLt over a cached bf16 W; fp32 weight/bias grads."""

    @staticmethod
    def forward(ctx, x, w, b, w16, res=None, blink=None):
        x = x.to(torch.bfloat16)
        x2 = x.reshape(-1, x.shape[-1])
        if b is not None:
            y = torch.addmm(b.to(torch.bfloat16), x2, w16.t())
        else:
            y = x2 @ w16.t()
        ctx.save_for_backward(x2, w16)
        ctx.has_b = b is not None
        ctx.shape = x.shape
        ctx.params = (w, b)  # flat-gradient direct-write targets (ops/grad_sink.py)
        ctx.res = res
        ctx.blink = blink
        return y.view(*x.shape[:-1], w16.shape[0])

    @staticmethod
    def backward(ctx, dy):
        x2, w16 = ctx.saved_tensors
        dy2 = dy.reshape(-1, dy.shape[-1]).to(torch.bfloat16)
        dx = None
        if ctx.needs_input_grad[0]:
            # + the residual branch's gradient of the same x (ResidualLink), in place: C += dY W
            # in the GEMM epilogue (out-of-place addmm copies C first)
            dx = _dx_residual(ctx.res, dy2, w16, ctx.shape)
        pw, pb = ctx.params
        dw = db = None
        if ctx.needs_input_grad[1]:
            tw = grad_sink.write_target(pw)
            dw = wgrad_f32(dy2, x2, out=tw)
            if tw is not None:
                grad_sink.done(pw)
                dw = None
        if ctx.has_b and ctx.needs_input_grad[2]:
            tb = grad_sink.write_target(pb)
            # a first contribution's region is zero; the attention backward's partial column
            # sums stand in for dY when linked (BiasGradLink)
            blink = ctx.blink
            src = blink.part if blink is not None and blink.part is not None else dy2
            db = dops.colsum(src, out=tb, accumulate=tb is not None)
            if blink is not None:
                blink.part = None
            if tb is not None:
                grad_sink.done(pb)
                db = None
        return dx, dw, db, None, None, None


def linear(x: torch.Tensor, w: torch.Tensor, b: Optional[torch.Tensor] = None,
           res: Optional[ResidualLink] = None, bias_link: Optional[BiasGradLink] = None) -> torch.Tensor:
    if use_hip(x):
        return _Linear16Fn.apply(x, w, b, weight_bf16(w), res, bias_link)
    return F.linear(x, w.to(x.dtype), None if b is None else b.to(x.dtype))


def _dx_residual(res: Optional[ResidualLink], dy2: torch.Tensor, w16: torch.Tensor, shape) -> torch.Tensor:
    """dX = dY W (+ the residual branch's gradient parked in ``res``, added in the GEMM epilogue)."""
    rg = res.grad if res is not None else None
    if rg is None:
        return (dy2 @ w16).view(shape)
    res.grad = None
    if rg.dtype == dy2.dtype and rg.is_contiguous():
        return rg.view(-1, rg.shape[-1]).addmm_(dy2, w16).view(shape)
    return torch.addmm(rg.reshape(-1, rg.shape[-1]).to(dy2.dtype), dy2, w16).view(shape)


def ffn(x: torch.Tensor, w1: torch.Tensor, b1: torch.Tensor, w2: torch.Tensor,
        res: Optional[ResidualLink] = None) -> torch.Tensor:
    """The transformer FFN without its output bias: gelu(x W1^T + b1) W2^T (the output bias
    is added by the following add_layernorm).  The bias + GELU pair runs as one kernel in
    each direction (bias_gelu / its backward); the hipBLASLt GELU_AUX_BIAS / DGELU_BGRAD
    epilogues that would fold them into the GEMMs have no gfx950 bf16 solutions in torch
    2.10's hipBLASLt (round-5 probe, docs/PERF.md), so no GEMM-epilogue arm is kept."""
    return linear(bias_gelu(linear(x, w1, res=res), b1), w2)


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

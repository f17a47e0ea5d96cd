"""Fused linear + bias + activation (K4) and L2 normalisation (K5).

GPU forward: ``csrc/kernels/dense.hip`` (MFMA bf16, fp32 accumulate, fused epilogue).
Backward: the activation mask is a HIP elementwise kernel; dx = dz W runs on the same
linear_act kernel with W^T as its weight, dW = dz^T x on linear_wgrad_kernel (rows split
into partial slabs, reduced by the column-sum kernel).  On the model shapes both are at or
below hipBLASLt's time (tools/dense_bwd_micro.py, host-timed: MLP 512x512 dgrad 45 vs
74 us, wgrad 51 vs 72 us; CDSSM page tower 26 / 39 vs 33 / 35-42 us, query tower 12 / 21 vs
24 / 41 us).  ``PAGEVEC_DENSE_BWD=lib`` keeps the library GEMMs.
"""
from __future__ import annotations

import os
from typing import Optional

import torch

from . import grad_sink
from . import reference as ref
from ._common import P, check, lib, ref_precision, stream, use_hip, use_hip_exact

_ACT = {"none": 0, "relu": 1, "gelu": 2, "tanh": 3}


class _LinearActFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, act):
        x2 = x.reshape(-1, x.shape[-1])
        if x2.dtype not in (torch.float32, torch.bfloat16):
            x2 = x2.float()
        x2 = x2.contiguous()
        M, K = x2.shape
        N = w.shape[0]
        wc = w.contiguous()
        y = torch.empty(M, N, dtype=torch.float32, device=x.device)
        xdt = 1 if x2.dtype == torch.bfloat16 else 0
        wdt = 1 if wc.dtype == torch.bfloat16 else 0
        check(lib().pv_linear_act(P(x2), xdt, P(wc), wdt, P(b) if b is not None else None, P(y), None, M, N, K, K, N,
                                  _ACT[act], stream(x.device)), "pv_linear_act")
        ctx.save_for_backward(x2, w, y if act in ("relu", "tanh") else None, b)
        ctx.act = act
        ctx.xshape = x.shape
        ctx.params = (w, b)  # flat-gradient direct-write targets (ops/grad_sink.py)
        return y.view(*x.shape[:-1], N)

    @staticmethod
    def backward(ctx, dy):
        x2, w, y, b = ctx.saved_tensors
        dy2 = dy.reshape(-1, dy.shape[-1]).contiguous().float()
        if ctx.act in ("relu", "tanh"):
            dz = torch.empty_like(dy2)
            check(lib().pv_act_bwd(P(y), P(dy2), P(dz), dy2.numel(), _ACT[ctx.act], stream(dy.device)), "pv_act_bwd")
        elif ctx.act == "none":
            dz = dy2
        else:  # gelu: recompute pre-activation (rare path; BERT uses torch GEMM + gelu kernel instead)
            pre = torch.nn.functional.linear(x2.float(), w.float(), b)
            with torch.enable_grad():
                pre.requires_grad_(True)
                g = torch.autograd.grad(torch.nn.functional.gelu(pre, approximate="tanh"), pre, dy2)[0]
            dz = g
        hipb = _HIP_BWD and dz.is_cuda
        xf = x2 if hipb else x2.float()  # the in-tree kernels stage fp32 or bf16 x directly
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            dxf = dgrad_hip(dz, w) if hipb else dz @ w.float()
            dx = dxf.view(ctx.xshape).to(x2.dtype)
        wg = wgrad_hip if hipb else _wgrad
        if ctx.needs_input_grad[1]:
            tw = grad_sink.write_target(ctx.params[0])  # straight into the flat gradient (ops/grad_sink.py)
            if tw is not None:
                wg(dz, xf, out=tw)
                grad_sink.done(ctx.params[0])
            else:
                dw = wg(dz, xf).to(w.dtype)
        if b is not None and ctx.needs_input_grad[2]:
            tb = grad_sink.write_target(ctx.params[1])
            if tb is not None:
                colsum(dz, out=tb, accumulate=True)  # first contribution: the region is zero
                grad_sink.done(ctx.params[1])
            else:
                db = colsum(dz)
        return dx, dw, db, None


_COLSUM_HIP = os.environ.get("PAGEVEC_COLSUM", "1") != "0"  # 0: torch reductions (A/B)
# dense backward GEMMs on the in-tree kernels (dgrad on linear_act with W^T, wgrad on
# linear_wgrad_kernel); "lib": hipBLASLt through torch (A/B, tools/dense_bwd_micro.py)
_HIP_BWD = os.environ.get("PAGEVEC_DENSE_BWD", "hip") != "lib"
_WG_TARGET = int(os.environ.get("PAGEVEC_WGRAD_WG", "512"))  # wgrad workgroups (row slices x tiles)


def _colsum_ok(x: torch.Tensor, C: int, ldx: int) -> bool:
    return _COLSUM_HIP and x.is_cuda and x.dtype in (torch.float32, torch.bfloat16)


def colsum(x: torch.Tensor, out: Optional[torch.Tensor] = None, accumulate: bool = False, scale=None, bias=None,
           act: str = "none", scale_is_len: bool = False) -> torch.Tensor:
    """Sum over the leading axis of x (R, ...) -> fp32 (...) on the HIP column-sum kernel
    (dense.hip::colsum_kernel): the bias gradients and split-K partial sums of the backward.
    ``accumulate``: add into ``out`` (a zeroed buffer or a flat-gradient region).
    ``scale`` (rows of the result) / ``bias`` (its last axis) / ``act``: fused epilogue
    act(scale * sum + bias) of the split-K forward (no accumulate)."""
    R = x.shape[0]
    tail = x.shape[1:]
    C = 1
    for d in tail:
        C *= int(d)
    epi = scale is not None or bias is not None or act != "none"
    x2 = x.reshape(R, C) if x.is_contiguous() else x.contiguous().reshape(R, C)
    if use_hip_exact(x) and _colsum_ok(x2, C, C) and (out is None or (out.is_contiguous() and out.dtype == torch.float32)):
        E = int(tail[-1]) if len(tail) else 1
        if epi:
            mode = 3 if (scale_is_len and scale is not None) else 2
        elif accumulate or R > 64:
            mode = 1
        else:
            mode = 0
        if out is None:
            out = (torch.zeros if mode == 1 else torch.empty)(tail, dtype=torch.float32, device=x.device)
        elif mode == 1 and not accumulate:
            out.zero_()
        sc = scale.float().contiguous() if scale is not None else None
        bb = bias.float().contiguous() if bias is not None else None
        check(lib().pv_colsum(P(x2), 1 if x2.dtype == torch.bfloat16 else 0, R, C, C, P(out), mode, P(sc), P(bb), E,
                              _ACT[act], stream(x.device)), "pv_colsum")
        return out
    if not epi and out is not None and not accumulate and out.dtype == torch.float32:
        return torch.sum(x, 0, dtype=torch.float32, out=out)
    y = torch.sum(x, 0, dtype=torch.float32)
    if epi:
        if scale is not None:
            sc = (1.0 / scale.float().clamp(min=1.0)) if scale_is_len else scale.float()
            y = y * sc.reshape(-1, *([1] * (y.dim() - 1)))
        if bias is not None:
            y = y + bias.float()
        y = _torch_act(y, act)
    if out is None:
        return y
    return out.add_(y) if accumulate else out.copy_(y)


def _torch_act(y: torch.Tensor, act: str) -> torch.Tensor:
    if act == "relu":
        return torch.relu(y)
    if act == "tanh":
        return torch.tanh(y)
    if act == "gelu":
        return torch.nn.functional.gelu(y, approximate="tanh")
    return y


def _wgrad(dz: torch.Tensor, xf: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """dz^T x split over the row axis into batched GEMMs (the single GEMM of a 150 x 300
    output over 16384 rows runs on a handful of workgroups: 126 us in the CDSSM profile).
    ``out``: fp32 destination (a flat-gradient view), overwritten."""
    from .transformer import _wgrad_splits

    T = dz.shape[0]
    sk = _wgrad_splits(T)
    if sk == 1:
        return torch.mm(dz.t(), xf, out=out)
    part = torch.bmm(dz.view(sk, T // sk, -1).transpose(1, 2), xf.view(sk, T // sk, -1))
    return colsum(part, out=out)


def wgrad_hip(dz: torch.Tensor, x: torch.Tensor, out: Optional[torch.Tensor] = None, tile: int = 0) -> torch.Tensor:
    """dW (N, K) = dz^T x on the in-tree kernel (dense.hip::linear_wgrad_kernel): dz (M, N) and
    x (M, K) fp32 or bf16, row-major; rows split over workgroups into fp32 partial slabs that
    the column-sum kernel reduces in a fixed order.  ``out``: fp32 destination (overwritten)."""
    M, N = dz.shape
    K = x.shape[1]
    dzc, xc = dz.contiguous(), x.contiguous()
    tile = tile or (128 if min(N, K) >= 256 else 64)
    tiles = -(-N // tile) * -(-K // tile)
    want = max(1, min(-(-_WG_TARGET // tiles), M // 256, 64))  # ~_WG_TARGET workgroups, >= 256 rows each
    rows = -(-(-(-M // want)) // 64) * 64
    ns = -(-M // rows)
    ws = torch.empty(ns, N, K, dtype=torch.float32, device=dz.device)
    check(lib().pv_linear_wgrad(P(dzc), 1 if dzc.dtype == torch.bfloat16 else 0, P(xc),
                                1 if xc.dtype == torch.bfloat16 else 0, P(ws), M, N, K, rows, tile, stream(dz.device)),
          "pv_linear_wgrad")
    if ns == 1:
        return ws[0] if out is None else out.copy_(ws[0])
    return colsum(ws, out=out)


def dgrad_hip(dz: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    """dx (M, K) = dz W on the forward kernel, fp32.  Small weights (<= 64k elements: the
    CDSSM head) are read transposed straight from W in the kernel's staging
    (pv_linear_dgrad); larger ones (the MLP's 512 x 512) go through one W^T copy, whose
    vector loads beat the strided ones (tools/dense_bwd_micro.py: 39 + 6 vs 56 us)."""
    M, N = dz.shape
    K = w.shape[1]
    dzc = dz.contiguous()
    zdt = 1 if dzc.dtype == torch.bfloat16 else 0
    dx = torch.empty(M, K, dtype=torch.float32, device=dz.device)
    if w.numel() <= 65536:
        wc = w.detach().contiguous()
        check(lib().pv_linear_dgrad(P(dzc), zdt, P(wc), 1 if wc.dtype == torch.bfloat16 else 0, P(dx), M, N, K,
                                    stream(dz.device)), "pv_linear_dgrad")
    else:
        wt = w.detach().t().contiguous()
        check(lib().pv_linear_act(P(dzc), zdt, P(wt), 1 if wt.dtype == torch.bfloat16 else 0, None, P(dx), None,
                                  M, K, N, N, K, 0, stream(dz.device)), "pv_linear_act(dgrad)")
    return dx


def gemm_f32(a: torch.Tensor, b: torch.Tensor, a_t: bool = False, b_t: bool = False,
             bias: Optional[torch.Tensor] = None, act: str = "none", out: Optional[torch.Tensor] = None,
             accumulate: bool = False, splits: int = 1) -> torch.Tensor:
    """op(a) @ op(b) [+ bias, act] in exact fp32 on the fp32 MFMA (dense.hip::gemm_f32_kernel), the
    dense layers' GEMM at the reference precision.  ``a_t`` / ``b_t``: the operand is stored
    transposed (read through strides, no copy).  ``splits`` > 1: split-K partial slabs reduced by
    the column-sum kernel (no epilogue: bias / act / accumulate need splits == 1)."""
    a, b = a.contiguous(), b.contiguous()
    if a.dtype != torch.float32 or b.dtype != torch.float32:
        raise TypeError("gemm_f32: fp32 operands")
    M, K = (a.shape[1], a.shape[0]) if a_t else a.shape
    Kb, N = (b.shape[1], b.shape[0]) if b_t else b.shape
    if K != Kb:
        raise ValueError(f"gemm_f32: inner dims {K} vs {Kb}")
    sam, sak = (1, M) if a_t else (K, 1)
    sbk, sbn = (1, K) if b_t else (N, 1)
    bb = bias.contiguous().float() if bias is not None else None
    if splits > 1 and (bias is not None or act != "none" or accumulate):
        raise ValueError("gemm_f32: split-K partials take no epilogue")
    if splits > 1:
        kper = -(-(-(-K // splits)) // 16) * 16
        ns = -(-K // kper)
        ws = torch.empty(ns, M, N, dtype=torch.float32, device=a.device)
        check(lib().pv_gemm_f32(P(a), sam, sak, P(b), sbk, sbn, None, P(ws), N, M, N, K, ns, 0, 0, stream(a.device)),
              "pv_gemm_f32")
        if ns > 1:
            return colsum(ws, out=out)
        part = ws[0]
        return part if out is None else out.copy_(part)
    if out is None:
        out = torch.empty(M, N, dtype=torch.float32, device=a.device)
    elif not (out.is_contiguous() and out.shape == (M, N) and out.dtype == torch.float32):
        raise ValueError("gemm_f32: out must be a contiguous fp32 (M, N) tensor")
    check(lib().pv_gemm_f32(P(a), sam, sak, P(b), sbk, sbn, P(bb), P(out), N, M, N, K, 1, _ACT[act], int(accumulate),
                            stream(a.device)), "pv_gemm_f32")
    return out


def _wgrad_splits_f32(M: int, N: int, K: int) -> int:
    tiles = -(-N // 64) * -(-K // 64)
    return max(1, min(64, -(-512 // tiles), M // 256))


class _LinearF32Fn(torch.autograd.Function):
    """Dense + activation at the reference precision (dtype="fp32"): forward, dgrad and wgrad on
    the fp32-MFMA GEMM, the activation backward and bias column sum on their fp32 kernels; the
    weight / bias gradients written straight into the flat gradient like _LinearActFn."""

    @staticmethod
    def forward(ctx, x, w, b, act):
        x2 = x.reshape(-1, x.shape[-1]).contiguous().float()
        wf = w.contiguous().float()
        y = gemm_f32(x2, wf, b_t=True, bias=b, act=act)
        ctx.save_for_backward(x2, wf, y if act in ("relu", "tanh") else None, b)
        ctx.act = act
        ctx.xshape = x.shape
        ctx.params = (w, b)
        return y.view(*x.shape[:-1], w.shape[0])

    @staticmethod
    def backward(ctx, dy):
        x2, wf, y, b = ctx.saved_tensors
        dy2 = dy.reshape(-1, dy.shape[-1]).contiguous().float()
        if ctx.act in ("relu", "tanh"):
            dz = torch.empty_like(dy2)
            check(lib().pv_act_bwd(P(y), P(dy2), P(dz), dy2.numel(), _ACT[ctx.act], stream(dy.device)), "pv_act_bwd")
        elif ctx.act == "none":
            dz = dy2
        else:  # gelu: the pre-activation recomputed on the same GEMM
            pre = gemm_f32(x2, wf, b_t=True, bias=b)
            with torch.enable_grad():
                pre.requires_grad_(True)
                dz = torch.autograd.grad(torch.nn.functional.gelu(pre, approximate="tanh"), pre, dy2)[0]
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            dx = gemm_f32(dz, wf).view(ctx.xshape)
        if ctx.needs_input_grad[1]:
            M, N = dz.shape
            sk = _wgrad_splits_f32(M, N, x2.shape[1])
            tw = grad_sink.write_target(ctx.params[0])
            if tw is not None:
                gemm_f32(dz, x2, a_t=True, out=tw, splits=sk)
                grad_sink.done(ctx.params[0])
            else:
                dw = gemm_f32(dz, x2, a_t=True, splits=sk)
        if b is not None and ctx.needs_input_grad[2]:
            tb = grad_sink.write_target(ctx.params[1])
            if tb is not None:
                colsum(dz, out=tb, accumulate=True)
                grad_sink.done(ctx.params[1])
            else:
                db = colsum(dz)
        return dx, dw, db, None


def linear_act(x: torch.Tensor, w: torch.Tensor, b: Optional[torch.Tensor], act: str = "relu") -> torch.Tensor:
    if ref_precision() and x.is_cuda:  # dtype="fp32": exact fp32 on the fp32 MFMA
        use_hip_exact(x)
        return _LinearF32Fn.apply(x, w, b, act)
    if use_hip(x, w):
        return _LinearActFn.apply(x, w, b, act)
    return ref.linear_act(x, w, b, act)


class _L2NormFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        x2 = x.reshape(-1, x.shape[-1]).contiguous().float()
        M, D = x2.shape
        y = torch.empty_like(x2)
        inv = torch.empty(M, dtype=torch.float32, device=x.device)
        # the cosine-softmax losses read the vectors as zero-padded bf16 rows (32-multiple
        # width): written by the same kernel, handed over as an attribute of the output
        DP = (D + 31) // 32 * 32
        ybf = torch.empty(M, DP, dtype=torch.bfloat16, device=x.device) if DP <= 192 else None
        check(lib().pv_l2norm_fwd(P(x2), P(y), P(inv), P(ybf), M, D, DP if ybf is not None else D, stream(x.device)),
              "pv_l2norm_fwd")
        ctx.save_for_backward(x2, y, inv)
        ctx.shape = x.shape
        out = y.view(x.shape)
        if ybf is not None and len(x.shape) == 2:
            out._pv_bf16 = ybf
        return out

    @staticmethod
    def backward(ctx, dy):
        x2, y, inv = ctx.saved_tensors
        M, D = x2.shape
        dy2 = dy.reshape(M, D)
        if dy2.dtype != torch.float32 or dy2.stride(1) != 1 or dy2.stride(0) < D:
            dy2 = dy2.contiguous().float()
        # row-strided gradients (the loss kernels' (n, DP) padded dQ / dD sliced to D) are read
        # in place: no copy kernel
        dx = torch.empty_like(x2)
        check(lib().pv_l2norm_bwd_ld(P(y), P(inv), P(x2), P(dy2), dy2.stride(0), P(dx), M, D, stream(dy.device)),
              "pv_l2norm_bwd_ld")
        return dx.view(ctx.shape)


def l2_normalize(x: torch.Tensor) -> torch.Tensor:
    if use_hip_exact(x):
        return _L2NormFn.apply(x)
    return ref.l2_normalize(x)


class _ChunkMeanFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, v, ids, C, CL):
        N, _, D = v.shape
        vc = v.contiguous().float()
        idc = ids.contiguous()
        out = torch.empty(N, D, dtype=torch.float32, device=v.device)
        scale = torch.empty(N, C, dtype=torch.float32, device=v.device)
        check(lib().pv_chunk_mean_fwd(P(vc), P(idc), N, C, CL, D, P(out), P(scale), stream(v.device)),
              "pv_chunk_mean_fwd")
        ctx.save_for_backward(scale)
        ctx.shape = (N, C, D)
        return out

    @staticmethod
    def backward(ctx, g):
        (scale,) = ctx.saved_tensors
        N, C, D = ctx.shape
        dv = torch.empty(N, C, D, dtype=torch.float32, device=g.device)
        check(lib().pv_chunk_mean_bwd(P(g.contiguous().float()), P(scale), N, C, D, P(dv), stream(g.device)),
              "pv_chunk_mean_bwd")
        return dv, None, None, None


def chunk_mean_pool(v: torch.Tensor, ids: torch.Tensor, chunk_len: int) -> torch.Tensor:
    """v (N, C, D) chunk vectors, ids (N, C * chunk_len) token ids (0 = padding) -> the mean of
    the non-empty chunks' vectors (N, D); a page with no non-empty chunk gets zeros.  GPU: one
    fused kernel per direction (chunkpool.hip); CPU: the torch expression."""
    N, C, D = v.shape
    if use_hip(v, ids) and ids.dtype == torch.int32 and C <= 64 and ids.shape[1] == C * chunk_len:
        return _ChunkMeanFn.apply(v, ids, C, int(chunk_len))
    live = (ids.reshape(N, C, chunk_len) != 0).any(dim=2).unsqueeze(2).to(v.dtype)
    return (v * live).sum(1) / live.sum(1).clamp(min=1.0)

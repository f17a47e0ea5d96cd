"""FP8 (OCP e4m3) linear layer: quantise -> fp8 MFMA GEMM -> dequant + bias + act.

Forward GEMMs run on ``v_mfma_f32_16x16x32_fp8_fp8`` (csrc/kernels/fp8.hip) with
per-tensor current scaling (amax of this step's activation; weights re-quantised once
per optimizer step through the model's compute cache).  Backward uses bf16 GEMMs
(hipBLASLt) on the unquantised tensors — the usual fp8-forward / bf16-backward recipe.
CPU: emulated with torch.float8_e4m3fn round-trips (same scaling rule).
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch

from ._common import P, check, lib, stream, use_hip

FP8_MAX = 448.0
AMAX_PARTS = 512  # fp8.hip::AMAX_PARTS
_ACT = {"none": 0, "relu": 1, "tanh": 3}


def quantize(x: torch.Tensor, with_bf16: bool = False):
    """fp32 tensor -> (uint8 e4m3 bytes, amax device scalar); with_bf16: also a bf16 copy of
    x written by the same pass (the operand of the bf16 weight-gradient GEMM)."""
    x = x.contiguous().float()
    if x.data_ptr() % 16:  # the quantiser reads 16-byte vectors
        x = x.clone()
    n = x.numel()
    if n % 4:
        raise ValueError("fp8 quantisation needs numel % 4 == 0")
    # per-block partial maxima + the scalar in one uninitialised buffer: no zero-fill launch
    ws = torch.empty(AMAX_PARTS + 1, dtype=torch.float32, device=x.device)
    amax = ws[AMAX_PARTS:]
    q = torch.empty(x.shape, dtype=torch.uint8, device=x.device)
    x16 = torch.empty(x.shape, dtype=torch.bfloat16, device=x.device) if with_bf16 else None
    check(lib().pv_amax_quant_fp8(P(x), n, P(ws), P(amax), P(q), P(x16), stream(x.device)), "pv_amax_quant_fp8")
    return (q, amax, x16) if with_bf16 else (q, amax)


def quantize_t(w: torch.Tensor, ldo: int):
    """fp32 (V, E) -> (e4m3 bytes (E, ldo): W^T zero-padded along V to ldo, amax device scalar):
    the K-contiguous B operand of the MX fp8 GEMM (gemm_mx8), per-tensor scale 448 / amax."""
    w = w.detach().contiguous().float()
    V, E = w.shape
    ws = torch.empty(AMAX_PARTS + 1, dtype=torch.float32, device=w.device)
    amax = ws[AMAX_PARTS:]
    out = torch.empty(E, ldo, dtype=torch.uint8, device=w.device)
    check(lib().pv_amax_quant_fp8_t(P(w), V, E, P(ws), P(amax), P(out), ldo, stream(w.device)), "pv_amax_quant_fp8_t")
    return out, amax


MX_BK = 128  # gemm_mx8.hip BK (bytes of K per tile): K operands are padded to a multiple of it


def mx8_ksplit(M: int, N: int, K: int) -> int:
    """K slices so that the 256 x 128 output tiles x slices cover the 256 CUs (one 96 KB-LDS
    workgroup per CU), with >= 8 K tiles per slice."""
    tiles = -(-M // 256) * -(-N // 128)
    ks = max(1, 256 // tiles)
    return max(1, min(ks, (K // MX_BK) // 8))


def gemm_mx8(a8: torch.Tensor, b8: torch.Tensor, alpha: float = 1.0, alpha_ptr: Optional[torch.Tensor] = None,
             ksplit: Optional[int] = None) -> torch.Tensor:
    """fp32 alpha * (*alpha_ptr) * a8 (M, K) . b8 (N, K)^T on the block-scaled fp8 MFMA
    (csrc/kernels/gemm_mx8.hip); e4m3 bytes, K % 128 == 0.  ksplit > 1 returns the (ksplit,
    M, N) fp32 partials (the caller's column-sum reduces them with its epilogue)."""
    M, K = a8.shape
    N = b8.shape[0]
    ks = mx8_ksplit(M, N, K) if ksplit is None else int(ksplit)
    out = torch.empty((ks, M, N) if ks > 1 else (M, N), dtype=torch.float32, device=a8.device)
    check(lib().pv_gemm_mx8(P(a8), a8.stride(0), P(b8), b8.stride(0), P(out), N, M, N, K, ks, M * N, None,
                            float(alpha), P(alpha_ptr) if alpha_ptr is not None else None, 0, 0,
                            stream(a8.device)), "pv_gemm_mx8")
    return out


def emulate_e4m3(x: torch.Tensor) -> torch.Tensor:
    """Round to the nearest OCP e4m3 value (saturating at +-448), as the GPU conversion."""
    return x.float().clamp(-FP8_MAX, FP8_MAX).to(torch.float8_e4m3fn).float()


def _emulate(x: torch.Tensor) -> torch.Tensor:
    """e4m3 round trip with per-tensor current scaling, as the HIP quantiser.  The backward
    is straight-through (identity), like the HIP path's bf16 backward GEMMs on the
    unquantised operands: a float8 cast has no autograd edge, so without the detach trick
    no gradient would reach x or w at all."""
    with torch.no_grad():
        a = x.abs().max().clamp(min=1e-12)
        s = FP8_MAX / a
        q = (x * s).clamp(-FP8_MAX, FP8_MAX).to(torch.float8_e4m3fn).float() / s
    return x + (q - x).detach() if x.requires_grad else q


class _FP8LinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, act, wq):
        x2 = x.reshape(-1, x.shape[-1]).contiguous().float()
        M, K = x2.shape
        N = w.shape[0]
        xq, ax, x16 = quantize(x2, with_bf16=True)  # x16: the wgrad operand (no fp32 copy saved)
        w8, aw = wq if wq is not None else quantize(w.detach())
        y = torch.empty(M, N, dtype=torch.float32, device=x.device)
        check(lib().pv_fp8_linear(P(xq), P(w8), P(ax), P(aw), P(b) if b is not None else None, P(y), None, M, N, K,
                                  _ACT[act], stream(x.device)), "pv_fp8_linear")
        ctx.save_for_backward(x16, y if act != "none" else None)
        ctx.act, ctx.xshape = act, x.shape
        ctx.params = (w, b)  # flat-gradient direct-write targets (ops/grad_sink.py)
        return y.view(*x.shape[:-1], N)

    @staticmethod
    def backward(ctx, dy):
        from . import dense as dops
        from . import grad_sink
        from .transformer import weight_bf16, wgrad_f32

        x16, y = ctx.saved_tensors
        w, b = ctx.params
        dz = dy.reshape(-1, dy.shape[-1]).contiguous().float()
        if y is not None:  # activation mask + the bf16 copy in one kernel
            dzm = torch.empty_like(dz)
            dzb = torch.empty(dz.shape, dtype=torch.bfloat16, device=dz.device)
            check(lib().pv_act_bwd2(P(y), P(dz), P(dzm), P(dzb), dz.numel(), _ACT[ctx.act], stream(dz.device)),
                  "pv_act_bwd2")
            dz = dzm
        else:
            dzb = dz.to(torch.bfloat16)
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            try:
                dx = torch.mm(dzb, weight_bf16(w), out_dtype=torch.float32)
            except (TypeError, RuntimeError, NotImplementedError):
                dx = (dzb @ weight_bf16(w)).float()
            dx = dx.view(ctx.xshape)
        if ctx.needs_input_grad[1]:
            tw = grad_sink.write_target(w)
            dw = wgrad_f32(dzb, x16, out=tw)  # split-K fp32, straight into the flat grad
            if tw is not None:
                grad_sink.done(w)
                dw = None
        if b is not None and ctx.needs_input_grad[2]:
            tb = grad_sink.write_target(b)
            db = dops.colsum(dz, out=tb, accumulate=tb is not None)
            if tb is not None:
                grad_sink.done(b)
                db = None
        return dx, dw, db, None, None


def fp8_linear(x: torch.Tensor, w: torch.Tensor, b: Optional[torch.Tensor], act: str = "none",
               wq: Optional[Tuple[torch.Tensor, torch.Tensor]] = None) -> torch.Tensor:
    """y = act(x @ w^T + b) with e4m3 operands and fp32 accumulation."""
    if use_hip(x, w):
        return _FP8LinearFn.apply(x, w, b, act, wq)
    y = torch.nn.functional.linear(_emulate(x.float()), _emulate(w.float()), b)
    return {"none": y, "relu": torch.relu(y), "tanh": torch.tanh(y)}[act]

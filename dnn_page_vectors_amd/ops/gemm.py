"""bf16 GEMM engine (csrc/kernels/gemm.hip) for the dense layers' plain and fused GEMMs.

``gemm(a, b, a_col, b_col)`` computes C = epilogue(alpha * A . B^T) with A logical [M][K]
and B logical [N][K]; ``a_col`` / ``b_col`` say the operand is STORED transposed (A as
[K][M], B as [K][N]), so all three GEMMs of a linear layer run without a transpose copy:

    forward  y  = x W^T      gemm(x, W)                       A row, B row
    dgrad    dx = dy W       gemm(dy, W, b_col=True)           A row, B col
    wgrad    dW = dy^T x     gemm(dy, x, a_col=True, b_col=True)

Epilogue in the kernel: per-column bias, relu / gelu(tanh) / tanh, fp32 or bf16 output,
beta = 1 accumulation (C += ...).  Few output tiles and a long K (weight gradients, the bag
GEMMs) run split-K: fp32 partial slabs reduced by the column-sum kernel, with the same
bias / activation epilogue there.

Requirements of the kernel: bf16 operands, 16-byte aligned, row strides multiples of 8
elements, K a multiple of 64, M (N) a multiple of 8 for a transposed A (B).  ``supported``
checks them; callers fall back to the library GEMM otherwise.

Status (round 4, measured, profiles/r4_gemm/): correct for every storage combination,
split-K and epilogue (tests/test_kernels_gpu.py::test_gemm_engine_*); with the grouped tile
order 0.5-1.2 PF/s, 60-90% of hipBLASLt on the same shapes.  The 8-phase schedule (v4) and
the staggered 4-phase one (v3) were exact but not faster and are gone; the model paths keep
the library GEMMs (``USE`` is empty).
"""
from __future__ import annotations

import os
from typing import Optional

import torch

from ._common import P, check, lib, stream

_ACT = {"none": 0, "relu": 1, "gelu": 2, "tanh": 3}
BM = BN = 256
BK = 64


def _ld(t: torch.Tensor) -> int:
    return t.stride(0)


def supported(a: torch.Tensor, b: torch.Tensor, a_col: bool, b_col: bool) -> bool:
    if not (a.is_cuda and b.is_cuda and a.dtype == torch.bfloat16 and b.dtype == torch.bfloat16):
        return False
    if a.dim() != 2 or b.dim() != 2 or a.stride(1) != 1 or b.stride(1) != 1:
        return False
    K = a.shape[0] if a_col else a.shape[1]
    M = a.shape[1] if a_col else a.shape[0]
    N = b.shape[1] if b_col else b.shape[0]
    if K % BK or (b.shape[0] if b_col else b.shape[1]) != K:
        return False
    if a.data_ptr() % 16 or b.data_ptr() % 16 or _ld(a) % 8 or _ld(b) % 8:
        return False
    return not ((a_col and M % 8) or (b_col and N % 8))


def auto_ksplit(M: int, N: int, K: int) -> int:
    """K slices so that tiles x slices fills the 256 CUs, each slice >= 8 K-tiles (512)."""
    tiles = -(-M // BM) * -(-N // BN)
    ks = 1
    while tiles * ks * 2 <= 512 and K // (BK * ks * 2) >= 8:
        ks *= 2
    return ks


_WS = {}


def gemm(a: torch.Tensor, b: torch.Tensor, a_col: bool = False, b_col: bool = False, *,
         out: Optional[torch.Tensor] = None, bias: Optional[torch.Tensor] = None, act: str = "none",
         alpha: float = 1.0, accumulate: bool = False, out_dtype: torch.dtype = torch.float32,
         ksplit: int = 0) -> torch.Tensor:
    """C (M, N) = act(alpha * A . B^T + bias) (+ C when ``accumulate``)."""
    M = a.shape[1] if a_col else a.shape[0]
    K = a.shape[0] if a_col else a.shape[1]
    N = b.shape[1] if b_col else b.shape[0]
    if not supported(a, b, a_col, b_col):
        raise ValueError(f"gemm: unsupported operands {tuple(a.shape)}/{a.dtype} col={a_col}, "
                         f"{tuple(b.shape)}/{b.dtype} col={b_col}")
    dev = a.device
    bf = bias.float().contiguous() if bias is not None else None
    ks = ksplit or auto_ksplit(M, N, K)
    if out is not None:
        out_dtype = out.dtype
    if accumulate and out_dtype != torch.float32 and ks > 1:
        ks = 1  # bf16 accumulation happens in the kernel epilogue (no split-K reduce for it)
    if out is None:
        out = (torch.zeros if (accumulate and ks > 1) else torch.empty)(M, N, dtype=out_dtype, device=dev)
    s = stream(dev)
    if ks == 1:
        check(lib().pv_gemm_bf16(P(a), _ld(a), int(a_col), P(b), _ld(b), int(b_col), P(out), out.stride(0), M, N, K,
                                 1, 0, P(bf), float(alpha), _ACT[act], int(accumulate),
                                 int(out_dtype == torch.bfloat16), s), "pv_gemm_bf16")
        return out
    ws = torch.empty(ks, M, N, dtype=torch.float32, device=dev)
    check(lib().pv_gemm_bf16(P(a), _ld(a), int(a_col), P(b), _ld(b), int(b_col), P(ws), N, M, N, K, ks, M * N,
                             None, float(alpha), 0, 0, 0, s), "pv_gemm_bf16")
    from . import dense as dops

    if out_dtype != torch.float32:
        r = dops.colsum(ws, bias=bf, act=act)
        out.copy_(r)
        return out
    if accumulate:
        if bias is not None or act != "none":
            raise ValueError("split-K accumulate takes no epilogue")
        return dops.colsum(ws, out=out, accumulate=True)
    if bias is not None or act != "none":
        out.copy_(dops.colsum(ws, bias=bf, act=act))
        return out
    return dops.colsum(ws, out=out)


ENABLED = os.environ.get("PAGEVEC_GEMM", "1") != "0"

# Which GEMMs of a linear layer go to the engine instead of hipBLASLt.  Measured
# (tools/gemm_engine_micro.py, profiles/r3_gemm_engine.md): the engine reaches 0.47-0.96 PF/s
# where the library reaches 0.75-1.48 PF/s on the same operands, so NONE by default;
# PAGEVEC_GEMM_USE=fwd,dgrad,wgrad routes them (A/B, fused-epilogue experiments).
_DEFAULT_USE = set()
USE = set(filter(None, os.environ.get("PAGEVEC_GEMM_USE", ",".join(sorted(_DEFAULT_USE))).split(",")))


def use(kind: str, a: torch.Tensor, b: torch.Tensor, a_col: bool = False, b_col: bool = False) -> bool:
    """Route GEMM ``kind`` (fwd / dgrad / wgrad / bag) to the engine?"""
    return ENABLED and kind in USE and supported(a, b, a_col, b_col)

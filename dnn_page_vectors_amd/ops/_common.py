"""Shared helpers for the op wrappers: backend selection, pointers, streams, checks."""
from __future__ import annotations

import contextlib
import logging
import os
from typing import Optional

import torch

from .. import _native

_FORCE = os.environ.get("PAGEVEC_BACKEND", "")  # "", "hip", "torch"


def set_backend(name: str) -> None:
    """Force the op backend: 'hip', 'torch' (eager baseline) or '' (auto)."""
    global _FORCE
    if name not in ("", "auto", "hip", "torch"):
        raise ValueError(name)
    _FORCE = "" if name == "auto" else name


def get_backend() -> str:
    return _FORCE or "auto"


_FP32_NOTED = [False]


@contextlib.contextmanager
def precision_scope(cfg):
    """Compute precision of a model's forward ops (``Configuration.dtype``).

    ``bf16`` (default): the HIP kernels — bf16 MFMA operands, fp32 accumulation, fp32 master
    weights and optimizer state.  ``fp32``: the reference's precision (Keras/Theano trains in
    fp32, dssm_cnn_v2/cnn_dssm_th.py:182) — inside this scope no bf16 HIP kernel runs: the CDSSM
    conv tower runs its fp32 HIP kernels (csrc/kernels/conv_pool_f32.hip, fp32 MFMA; see
    ``ref_precision``), the dense layers the fp32-MFMA GEMM (dense.hip gemm_f32_kernel), the
    L2 normalisation / explicit loss / column sums / activation backward their fp32 kernels
    (``use_hip_exact``); the remaining ops (in-batch losses, transformer and LSTM towers, bag
    GEMMs) their fp32 PyTorch implementation.  The fused Adam kernel is fp32 already.  CPU runs
    are fp32 either way."""
    global _FORCE
    if getattr(cfg, "dtype", "bf16") != "fp32" or _FORCE == "torch":
        yield
        return
    if not _FP32_NOTED[0]:
        logging.getLogger(__name__).info("dtype=fp32: reference-precision ops (fp32 conv kernels, no bf16 HIP kernels)")
        _FP32_NOTED[0] = True
    prev, _FORCE = _FORCE, "torch"
    _REF_PREC[0] += 1
    try:
        yield
    finally:
        _FORCE = prev
        _REF_PREC[0] -= 1


_REF_PREC = [0]
# 0: dtype="fp32" runs the conv tower as PyTorch ops too (conv1d materialises (N, F, L); A/B)
F32_NATIVE = os.environ.get("PAGEVEC_F32_NATIVE", "1") != "0"


def ref_precision() -> bool:
    """Inside a dtype="fp32" precision scope with the native fp32 kernels enabled."""
    return _REF_PREC[0] > 0 and F32_NATIVE


def use_hip_exact(*tensors: torch.Tensor) -> bool:
    """``use_hip`` for kernels whose arithmetic is fp32 end to end (no bf16 operand: L2
    normalisation, column sums, activation backward, the explicit loss): inside a dtype="fp32"
    scope they run too, beside the fp32-MFMA dense / conv kernels (``ref_precision``)."""
    if ref_precision():
        if any(t is not None and t.is_cuda for t in tensors):
            _native.hip(required=True)
            return True
        return False
    return use_hip(*tensors)


def use_hip(*tensors: torch.Tensor) -> bool:
    """HIP kernels for CUDA tensors (required: raises if the library is missing), torch on CPU."""
    if _FORCE == "torch":
        return False
    on_gpu = any(t is not None and t.is_cuda for t in tensors)
    if _FORCE == "hip" and not on_gpu:
        raise RuntimeError("backend 'hip' requested for CPU tensors")
    if on_gpu:
        _native.hip(required=True)
        return True
    return False


def lib():
    return _native.hip(required=True)


def stream(device: Optional[torch.device] = None) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def P(t: Optional[torch.Tensor]) -> Optional[int]:
    return None if t is None else t.data_ptr()


def check(rc: int, name: str) -> None:
    if rc != 0:
        raise RuntimeError(f"{name} failed with status {rc}")


def need(t: torch.Tensor, dtype: torch.dtype, name: str, ndim: Optional[int] = None) -> torch.Tensor:
    if t.dtype != dtype:
        raise TypeError(f"{name}: expected {dtype}, got {t.dtype}")
    if ndim is not None and t.dim() != ndim:
        raise ValueError(f"{name}: expected {ndim}-D, got shape {tuple(t.shape)}")
    return t.contiguous()

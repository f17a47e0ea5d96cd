"""Shared helpers for the op wrappers: backend selection, pointers, streams, checks."""
from __future__ import annotations

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

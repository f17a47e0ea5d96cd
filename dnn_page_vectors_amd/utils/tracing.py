"""roctx ranges around the phases of a step (featurize / H2D / forward / backward /
allreduce / optimizer), visible in ``rocprofv3 --marker-trace`` timelines.

Disabled unless ``PAGEVEC_ROCTX=1`` (the markers are host calls on the hot path).
torch's nvtx shim maps to roctx on ROCm builds.
"""
from __future__ import annotations

import os
from contextlib import contextmanager

_ENABLED = os.environ.get("PAGEVEC_ROCTX", "0") == "1"


def enable(flag: bool = True) -> None:
    global _ENABLED
    _ENABLED = flag


def range_push(name: str) -> None:
    if _ENABLED:
        try:
            import torch

            torch.cuda.nvtx.range_push(name)
        except Exception:
            pass


def range_pop() -> None:
    if _ENABLED:
        try:
            import torch

            torch.cuda.nvtx.range_pop()
        except Exception:
            pass


@contextmanager
def trace_range(name: str):
    range_push(name)
    try:
        yield
    finally:
        range_pop()

"""Deterministic reduction mode ("two runs give equal loss with deterministic
reduction mode").

The fast GPU training step is reproducible only to rounding: the sparse conv backward
(dW / db per sample split, the embedding-table reduce's run-boundary flushes, the query
tower's rows reduce), the column-sum kernel's row splits and the gradient-norm kernel
combine partial sums with float atomics, whose result depends on arrival order.  With
``set_deterministic(True)`` (or ``Configuration.deterministic``):

* those kernels add int64 fixed-point values instead (resolution 2^-40, saturating at
  +-2^23; ``csrc/kernels/common.h::fx_add``): integer addition is associative, so the total
  does not depend on arrival order, and one ordered pass (``det.hip::fx_flush_kernel``)
  adds it into the float gradient;
* the column-sum kernel uses one row split (a single atomic per column and launch), the
  MLP embedding bag's sparse backward sends its run-boundary sums through the fixed-point
  buffer too, and torch's own ops use their deterministic algorithms
  (``torch.use_deterministic_algorithms``: the BERT token-embedding ``index_add_``);
* a training step runs on ONE HIP stream (no query-tower or dW side streams), and
  ``Trainer`` does not capture hipGraphs (the fixed-point buffer may grow between steps).

Everything else on the CDSSM step (fused conv forward, dense / L2 kernels, the loss kernels'
fixed-order split sums, the radix sort, Adam) is order-free already.  Cost: the extra
memset + flush per accumulating launch (the 30k x 100 table: 24 MB of int64 per reduce).
CPU training is always deterministic (tests/test_determinism.py).
"""
from __future__ import annotations

from .. import _native

_ON = [False]
_TORCH_PREV = [None]  # torch's deterministic-algorithm flags before this module switched them on


def set_deterministic(on: bool = True):
    """Switch the mode; returns the previous state (for ``restore``).  Switching it off also
    gives torch's deterministic-algorithm flags back the values they had before it was on."""
    import torch
    import torch.utils.deterministic as _tud

    prev = (_ON[0], torch.are_deterministic_algorithms_enabled(),
            torch.is_deterministic_algorithms_warn_only_enabled(), _tud.fill_uninitialized_memory)
    _ON[0] = bool(on)
    if not torch.cuda.is_available():  # CPU training is deterministic without the kernels' mode
        return prev
    # the few torch ops on the training paths (the BERT token-embedding index_add_) switch to
    # their deterministic implementations; uninitialised memory is NOT NaN-filled (every
    # kernel output is fully written; padded operands are allocated zeroed)
    if on:
        if _TORCH_PREV[0] is None:
            _TORCH_PREV[0] = prev[1:]
        torch.use_deterministic_algorithms(True, warn_only=True)
        _tud.fill_uninitialized_memory = False
    elif _TORCH_PREV[0] is not None:
        algos, warn_only, fill = _TORCH_PREV[0]
        _TORCH_PREV[0] = None
        torch.use_deterministic_algorithms(algos, warn_only=warn_only)
        _tud.fill_uninitialized_memory = fill
    lib = _native.hip(required=False)
    if lib is not None:
        lib.pv_set_deterministic(1 if on else 0)
    return prev


def restore(prev) -> None:
    """Undo ``set_deterministic``: the native flag and torch's global flags as they were."""
    import torch
    import torch.utils.deterministic as _tud

    on, algos, warn_only, fill = prev
    _ON[0] = bool(on)
    if not on:
        _TORCH_PREV[0] = None
    if torch.cuda.is_available():
        torch.use_deterministic_algorithms(algos, warn_only=warn_only)
        _tud.fill_uninitialized_memory = fill
        lib = _native.hip(required=False)
        if lib is not None:
            lib.pv_set_deterministic(1 if on else 0)


def enabled() -> bool:
    return _ON[0]


def ensure(on: bool) -> None:
    """Put the process-wide mode in state ``on`` if it is not (a Trainer calls this before
    every step, so trainers with different settings in one process each run in their own
    mode whatever order they were built or stepped in)."""
    if _ON[0] != bool(on):
        set_deterministic(on)

"""Direct parameter-gradient writes into the flat gradient buffer.

``FlatParams`` (ops/optim.py) makes every ``param.grad`` a view of one flat fp32 buffer.
A custom autograd op that returns its weight gradient makes autograd's AccumulateGrad
node run ``param.grad += dW``: one extra elementwise kernel per parameter, plus the
temporary dW (and, for bf16 GEMM outputs, a bf16 -> fp32 conversion).  In the MLP-DSSM
step those kernels were 12 adds + 3 conversions ~ 0.2 ms of a 1.6 ms step; in BERT they
are ~200 adds.  The HIP-path ops therefore ask this module for the parameter's flat-grad
view and write the gradient there themselves (GEMM ``out=``, atomically-accumulating
kernels), returning ``None`` to autograd for that input:

* ``accum_target(p)``  — for kernels that *add* into their output (the conv backward's
  atomics): always valid while ``p.grad`` is the flat view;
* ``write_target(p)``  — for ops that *overwrite* their output: valid only for the first
  gradient contribution to ``p`` since ``FlatParams.zero_grad`` (a parameter used twice,
  or micro-batch accumulation without a zero_grad, falls back to the autograd return);
* ``done(p)``          — mark ``p`` written this step and fire the data-parallel bucket
  hooks (parallel/ddp.py) that ``register_post_accumulate_grad_hook`` would have fired.

Data parallel: a bucket's all-reduce is launched from ``done`` as soon as all its
parameters are written.  A parameter that ALSO receives a gradient from another node of
the same graph would get that later contribution added while its bucket is already in
flight, so ``mark_multi_use(loss, flat)`` walks the autograd graph once (per input shape)
before backward and excludes every parameter with more than one consumer edge.
(Without data parallelism the ``written`` set alone keeps every case exact.)

``PAGEVEC_DIRECT_GRAD=0`` disables direct writes (A/B measurement, debugging).
"""
from __future__ import annotations

import os
from typing import Callable, Optional

import torch

ENABLED = os.environ.get("PAGEVEC_DIRECT_GRAD", "1") != "0"


def _flat(p: torch.Tensor):
    return getattr(p, "_pv_flat", None) if ENABLED else None


def accum_target(p: Optional[torch.Tensor]) -> Optional[torch.Tensor]:
    if p is None or torch.is_grad_enabled():  # create_graph backward: keep autograd's path
        return None
    f = _flat(p)
    if f is None or p.grad is None or p.grad.dtype != torch.float32 or not f.owns_grad(p) or id(p) in f.multi:
        return None
    return p.grad


def write_target(p: Optional[torch.Tensor]) -> Optional[torch.Tensor]:
    g = accum_target(p)
    if g is None or id(p) in p._pv_flat.written:
        return None
    return g


def done(p: torch.Tensor) -> None:
    p._pv_flat.written.add(id(p))
    for h in getattr(p, "_pv_sink_hooks", ()):
        h(p)


def add_hook(p: torch.Tensor, fn: Callable[[torch.Tensor], None]) -> Callable[[], None]:
    """Register ``fn(p)`` to run when an op writes p's gradient directly; returns a remover."""
    hooks = list(getattr(p, "_pv_sink_hooks", ()))
    hooks.append(fn)
    p._pv_sink_hooks = tuple(hooks)

    def remove():
        p._pv_sink_hooks = tuple(h for h in getattr(p, "_pv_sink_hooks", ()) if h is not fn)
    return remove


def mark_multi_use(root: torch.Tensor, flat) -> int:
    """Count the autograd edges into each parameter's AccumulateGrad node under ``root``;
    parameters of ``flat`` reached more than once are excluded from direct writes.
    Returns the number of such parameters."""
    counts = {}
    seen = set()
    stack = [root.grad_fn]
    while stack:
        fn = stack.pop()
        if fn is None or fn in seen:
            continue
        seen.add(fn)
        for nxt, _ in fn.next_functions:
            if nxt is None:
                continue
            var = getattr(nxt, "variable", None)
            if var is not None:  # AccumulateGrad
                counts[id(var)] = counts.get(id(var), 0) + 1
            else:
                stack.append(nxt)
    ids = {id(p) for _, p in flat.named}
    flat.multi = {i for i, c in counts.items() if c > 1 and i in ids}
    return len(flat.multi)

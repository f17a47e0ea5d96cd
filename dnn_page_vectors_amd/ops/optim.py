"""Flat-buffer parameter store + fused Adam (K8).

``FlatParams`` moves every parameter of a module into ONE contiguous fp32 buffer
(parameters become views), with a parallel flat gradient buffer that autograd
accumulates into (``param.grad`` are views as well).  Consequences:

* the optimizer is one streaming kernel over the flat buffers (csrc/kernels/optim.hip);
* data-parallel gradient all-reduce operates on contiguous buckets of the flat
  gradient (parallel/ddp.py) — no per-tensor packing;
* checkpoints / broadcast are single tensors.

Keras-1 Adam semantics by default (``torch_style=False``), see optim.hip.
"""
from __future__ import annotations

import math
from typing import Dict, Iterable, List, Optional, Sequence, Tuple

import torch

from . import reference as ref
from ._common import P, check, lib, stream, use_hip

ALIGN = 64  # elements: 256-byte aligned parameter starts


class FlatParams:
    def __init__(self, params: Iterable[Tuple[str, torch.nn.Parameter]], device: Optional[torch.device] = None):
        self.named: List[Tuple[str, torch.nn.Parameter]] = [(n, p) for n, p in params if p.requires_grad]
        if not self.named:
            raise ValueError("no trainable parameters")
        dev = device or self.named[0][1].device
        self.offsets: Dict[str, Tuple[int, int, torch.Size]] = {}
        off = 0
        for n, p in self.named:
            self.offsets[n] = (off, p.numel(), p.shape)
            off += (p.numel() + ALIGN - 1) // ALIGN * ALIGN
        self.numel = off
        self.data = torch.zeros(off, dtype=torch.float32, device=dev)
        self.grad = torch.zeros(off, dtype=torch.float32, device=dev)
        # direct gradient writes (ops/grad_sink.py): params written this step, flat-grad
        # addresses, and a hook marking params that autograd's AccumulateGrad wrote
        self.written = set()
        self.multi = set()  # params with several consumers (grad_sink.mark_multi_use)
        self._gptr: Dict[int, int] = {}
        self._hooks = []
        for n, p in self.named:
            o, k, shp = self.offsets[n]
            self.data[o:o + k].copy_(p.data.reshape(-1).float())
            p.data = self.data[o:o + k].view(shp)
            p.grad = self.grad[o:o + k].view(shp)
            self._gptr[id(p)] = p.grad.data_ptr()
            p._pv_flat = self
            self._hooks.append(p.register_post_accumulate_grad_hook(self._mark))

    def _mark(self, p) -> None:
        self.written.add(id(p))

    def owns_grad(self, p) -> bool:
        return p.grad is not None and self._gptr.get(id(p)) == p.grad.data_ptr()

    def zero_grad(self, skip: Sequence[Tuple[int, int]] = ()) -> None:
        """Zero the gradient buffer; ``skip``: sorted [lo, hi) element ranges left alone (the
        sparse-gradient tables, which zero only their touched rows: parallel/sparse_rows.py)."""
        if not skip:
            self.grad.zero_()
        else:
            pos = 0
            for lo, hi in skip:
                if lo > pos:
                    self.grad[pos:lo].zero_()
                pos = max(pos, hi)
            if pos < self.numel:
                self.grad[pos:].zero_()
        self.written.clear()

    def reattach_grads(self) -> None:
        """Re-point param.grad at the flat buffer (if something replaced them)."""
        for n, p in self.named:
            o, k, shp = self.offsets[n]
            g = self.grad[o:o + k].view(shp)
            if p.grad is None or p.grad.data_ptr() != g.data_ptr():
                if p.grad is not None:
                    g.copy_(p.grad)
                p.grad = g

    def state_dict(self) -> Dict[str, torch.Tensor]:
        return {n: self.data[o:o + k].view(shp) for n, (o, k, shp) in self.offsets.items()}


class FlatAdam:
    def __init__(self, flat: FlatParams, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8,
                 weight_decay: float = 0.0, torch_style: bool = False, lazy: Optional[Iterable[str]] = None,
                 mirror: Optional[Iterable[str]] = None, sparse=None, warmup: int = 0):
        """lazy: names of 2-D embedding tables updated LazyAdam-style — a row whose gradient is
        all zero this step (none of its tokens in the batch) keeps its weights and moments
        (optim.hip::adam_lazy_rows_kernel; the step then streams ~4 B instead of 28 B per
        untouched parameter, which is what makes word-level vocabularies of millions of rows
        cheap).  Default: dense Adam everywhere (Keras parity).

        mirror: names of parameters whose bf16 compute copy the update kernel writes in the
        same pass (``mirror_for(p)``): the forward's bf16 operands (MLP embedding tables,
        BERT projection weights) then need no per-step cast kernel."""
        self.flat = flat
        # sparse-gradient tables (parallel/sparse_rows.py): LazyAdam over their step's candidate
        # rows only (pv_adam_rows); on the CPU they are lazy tables over the whole table
        self.sparse = sparse
        sparse_names = set(sparse.tables) if sparse is not None else set()
        self._sparse_off = {sparse.tables[n].off: sparse.tables[n] for n in sparse_names}
        # [(offset, numel, row_len)] sorted by offset; rows of 4k floats (16-byte aligned)
        self.lazy: List[Tuple[int, int, int]] = []
        for name in sorted(set(lazy or ()) | sparse_names):
            o, k, shp = flat.offsets[name]
            if len(shp) == 2 and shp[1] % 4 == 0 and shp[1] <= 1024:
                self.lazy.append((o, k, int(shp[1])))
        self.lazy.sort()
        # ONE bf16 copy of the whole flat buffer, written by the same (single) update launch;
        # the named parameters' mirrors are views of it
        self.mirror16: Optional[torch.Tensor] = None
        self.mirrors: Dict[str, torch.Tensor] = {}
        if mirror and use_hip(flat.data):
            self.mirror16 = flat.data.detach().to(torch.bfloat16)
            named = dict(flat.named)
            for name in mirror:
                o, k, shp = flat.offsets[name]
                p = named[name]
                self.mirrors[name] = p._pv_mirror = self.mirror16[o:o + k].view(shp)
                p._pv_mirror_owner = flat
            flat.mirror_gen = _generation()  # mirrors equal the weights as of this generation
        self.lr, self.b1, self.b2, self.eps, self.wd = lr, betas[0], betas[1], eps, weight_decay
        self.torch_style = torch_style
        self.m = torch.zeros_like(flat.data)
        self.v = torch.zeros_like(flat.data)
        self.step_count = 0
        # the step count also lives on the device: the HIP update reads (and advances) it,
        # so a captured training step replays with the right bias corrections
        # t_dev = {step, linear warmup steps} (optim.hip warmup_scale)
        self.warmup = int(warmup)
        self.t_dev = torch.tensor([0.0, float(self.warmup)], dtype=torch.float32, device=flat.data.device)

    def step(self, skip_flag: Optional[torch.Tensor] = None) -> None:
        """One update. ``skip_flag``: device scalar; non-zero => the kernel skips (NaN guard)."""
        self.step_count += 1
        t = self.step_count
        lr = self.lr * (min(1.0, t / self.warmup) if self.warmup > 0 else 1.0)  # host paths
        if use_hip(self.flat.data):
            if self.lazy or self.mirrors or self.sparse is not None:
                self._step_segments(skip_flag)
                # the trainer bumps the generation right after the step: the mirrors hold
                # exactly the weights of that next generation
                if self.mirrors:
                    self.flat.mirror_gen = _generation() + 1
                return
            check(lib().pv_adam_dev(P(self.flat.data), P(self.flat.grad), P(self.m), P(self.v), self.flat.numel,
                                    P(self.t_dev), self.lr, self.b1, self.b2, self.eps, self.wd,
                                    int(self.torch_style), P(skip_flag), stream(self.flat.data.device)), "pv_adam_dev")
            return
        if skip_flag is not None and float(skip_flag) != 0.0:
            return
        keep = []
        for o, k, rl in self.lazy:  # CPU: dense update, then restore the untouched rows
            untouched = (self.flat.grad[o:o + k].view(-1, rl) == 0).all(1)
            keep.append((o, k, rl, untouched, [t[o:o + k].view(-1, rl)[untouched].clone()
                                                for t in (self.flat.data, self.m, self.v)]))
        with torch.no_grad():
            g = self.flat.grad + self.wd * self.flat.data if self.wd else self.flat.grad
            if self.torch_style:
                self.m.mul_(self.b1).add_(g, alpha=1 - self.b1)
                self.v.mul_(self.b2).addcmul_(g, g, value=1 - self.b2)
                bc1 = 1 - self.b1 ** t
                bc2 = 1 - self.b2 ** t
                self.flat.data.addcdiv_(self.m, (self.v.sqrt() / math.sqrt(bc2)).add_(self.eps), value=-lr / bc1)
            else:
                ref.adam_keras_([self.flat.data], [g], [self.m], [self.v], t, lr, self.b1, self.b2, self.eps)
            for o, k, rl, untouched, saved in keep:
                for tt, sv in zip((self.flat.data, self.m, self.v), saved):
                    tt[o:o + k].view(-1, rl)[untouched] = sv

    def _step_segments(self, skip_flag: Optional[torch.Tensor]) -> None:
        """Device step count +1, then dense updates of the gaps between lazy tables and lazy
        row updates of the tables (all reading the device counter: hipGraph-replayable)."""
        L_ = lib()
        s = stream(self.flat.data.device)
        check(L_.pv_step_inc(P(self.t_dev), s), "pv_step_inc")
        if not hasattr(self, "_segs"):
            pos = 0
            segs = []
            for o, k, rl in self.lazy:
                if o > pos:
                    segs.append((pos, o - pos, 0))
                segs.append((o, k, rl))
                pos = o + (k + 63) // 64 * 64
            if pos < self.flat.numel:
                segs.append((pos, self.flat.numel - pos, 0))
            self._segs = segs
        esz = self.flat.data.element_size()
        base = [t.data_ptr() for t in (self.flat.data, self.flat.grad, self.m, self.v)]
        m16 = self.mirror16
        for o, n, rl in self._segs:
            ptrs = [b + o * esz for b in base]
            mp = m16.data_ptr() + 2 * o if m16 is not None else None
            t = self._sparse_off.get(o) if rl else None
            if t is not None:  # sparse table: only this step's candidate rows
                rows = self.sparse.candidate_rows(t)
                check(L_.pv_adam_rows(ptrs[0], ptrs[1], ptrs[2], ptrs[3], rl, P(rows), rows.numel(), P(self.t_dev),
                                      self.lr, self.b1, self.b2, self.eps, self.wd, int(self.torch_style),
                                      P(skip_flag), mp, s), "pv_adam_rows")
                continue
            check(L_.pv_adam_seg(ptrs[0], ptrs[1], ptrs[2], ptrs[3], n, rl, P(self.t_dev), self.lr, self.b1, self.b2,
                                 self.eps, self.wd, int(self.torch_style), P(skip_flag), mp, s), "pv_adam_seg")

    def note_external_step(self) -> None:
        """A replayed hipGraph ran this optimizer's captured update (mirrors included)."""
        if self.mirrors:
            self.flat.mirror_gen = _generation() + 1

    def refresh_mirrors(self) -> None:
        """Re-cast the bf16 mirrors from the fp32 weights (after a checkpoint load / broadcast)."""
        if self.mirror16 is not None:
            self.mirror16.copy_(self.flat.data)
            self.flat.mirror_gen = _generation()

    def state_dict(self) -> Dict[str, object]:
        return {"m": self.m, "v": self.v, "step": self.step_count, "lr": self.lr}

    def load_state_dict(self, d: Dict[str, object]) -> None:
        self.m.copy_(d["m"])
        self.v.copy_(d["v"])
        self.step_count = int(d["step"])
        self.t_dev[0] = float(self.step_count)


def _generation() -> int:
    from ..models.base import _GENERATION

    return _GENERATION[0]


def mirror_for(p: torch.Tensor) -> Optional[torch.Tensor]:
    """The bf16 copy of ``p`` the optimizer wrote with its last update, if it is current
    (FlatAdam(mirror=...)); None -> the caller casts.  A generation bump that did not
    follow a mirrored step (checkpoint load, broadcast) makes it stale until the next step
    or ``refresh_mirrors``."""
    m = getattr(p, "_pv_mirror", None)
    if m is None or getattr(p._pv_mirror_owner, "mirror_gen", -1) != _generation():
        return None
    return m


def grad_sumsq_and_finite(flat_grad: torch.Tensor) -> torch.Tensor:
    """Device tensor [sum g^2, nonfinite_flag] without a host sync.  (A fill-free variant that
    finished the sums in the workgroup taking the last ticket of an agent-scope counter measured
    13 -> 35-50 us per call: every workgroup's release fence writes back its XCD's L2;
    profiles/r6/sumsq/.)"""
    out = torch.zeros(2, dtype=torch.float32, device=flat_grad.device)
    if use_hip(flat_grad):
        check(lib().pv_sumsq(P(flat_grad), flat_grad.numel(), P(out), stream(flat_grad.device)), "pv_sumsq")
        return out
    finite = torch.isfinite(flat_grad)
    out[0] = torch.where(finite, flat_grad, torch.zeros_like(flat_grad)).pow(2).sum()
    out[1] = (~finite).any().float()
    return out

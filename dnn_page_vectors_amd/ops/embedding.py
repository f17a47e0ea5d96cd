"""Embedding bag (sum / mean of token rows) for the DSSM MLP tower, and the device
trigram hasher (K0).

Two execution plans for ``bag = scale * onehot_counts(ids) @ W``:

* ``gather``  — HIP kernel gathers W rows per token (bf16 rows, one wave per bag); best for
  short bags (queries) and inference;
* ``counts``  — HIP kernel builds the dense count matrix C (N x V, bf16), then one
  hipBLASLt GEMM C @ W on the matrix cores; the backward is the GEMM C^T @ dY (no
  scatter atomics at all).  For 2k-token pages at V = 30k, E = 512 this is ~0.13 TFLOP
  of MFMA instead of ~8 GB of row gathers (fwd) + ~16 GB of float atomics (bwd).

The backward always uses the counts GEMM.  CPU: plain torch.
"""
from __future__ import annotations

from typing import Optional

import torch

from . import grad_sink
from . import reference as ref
from ._common import P, check, lib, stream, use_hip


_HIST_MAX = 38912  # csrc/kernels/embedding.hip HIST_MAX


def _counts(ids: torch.Tensor, V: int, pad: int):
    N, L = ids.shape
    ldc = (V + 63) // 64 * 64
    small = ldc <= _HIST_MAX  # LDS-histogram kernel writes every element itself (ldc % 64 == 0)
    C = (torch.empty if small else torch.zeros)(N, ldc, dtype=torch.bfloat16, device=ids.device)
    lens = torch.empty(N, dtype=torch.float32, device=ids.device)
    check(lib().pv_bag_counts(P(ids), P(C), P(lens), N, L, V, ldc, pad, int(not small), stream(ids.device)),
          "pv_bag_counts")
    return C, lens


def _counts_gemm(C: torch.Tensor, W16: torch.Tensor) -> torch.Tensor:
    """C (N, V) @ W16 (V, E) in fp32.  The (N, E) output has only (N/256)(E/256) = 32 tiles for
    the MLP page bags (N 4096, E 512) over a 30000-long reduction, so the single GEMM runs on
    a fraction of the CUs; split V into 8 batched fp32-output GEMMs and sum the partials:
    0.293 -> 0.148 ms (tools/bag_gemm_micro.py), and the result is no longer rounded to bf16."""
    N, V = C.shape
    E = W16.shape[1]
    sk = next((k for k in (8, 4, 2) if V % k == 0 and V // k >= 2048), 1)
    if sk > 1 and N * E <= 8 * 1024 * 1024:
        try:
            Cb = C.unflatten(1, (sk, V // sk)).transpose(0, 1)
            return torch.bmm(Cb, W16.reshape(sk, V // sk, E), out_dtype=torch.float32).sum(0)
        except (TypeError, RuntimeError, NotImplementedError):
            pass
    return (C @ W16).float()


class _BagFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, ids, W, W16, pad, mean, plan):
        ids = ids.to(torch.int32).contiguous()
        N, L = ids.shape
        V, E = W.shape
        C, lens = _counts(ids, V, pad)
        scale = (1.0 / lens.clamp(min=1.0)) if mean else torch.ones_like(lens)
        if plan == "gather":
            out = torch.empty(N, E, dtype=torch.float32, device=ids.device)
            check(lib().pv_embedding_bag(P(ids), P(W16), P(out), None, N, L, E, V, pad, int(mean),
                                         stream(ids.device)), "pv_embedding_bag")
        else:
            out = _counts_gemm(C[:, :V], W16) * scale[:, None]
        ctx.save_for_backward(C, scale)
        ctx.V = V
        ctx.W = W  # the parameter itself (its flat-gradient view is the direct-write target)
        return out

    @staticmethod
    def backward(ctx, g):
        C, scale = ctx.saved_tensors
        gs = (g.float() * scale[:, None]).to(torch.bfloat16)
        Ct = C[:, :ctx.V].t()
        if ctx.needs_input_grad[1]:
            W = ctx.W
            tw = grad_sink.write_target(W)  # fp32-output GEMM straight into the flat gradient
            if tw is not None:
                try:
                    torch.mm(Ct, gs, out_dtype=torch.float32, out=tw)
                except (TypeError, RuntimeError, NotImplementedError):
                    tw.copy_(Ct @ gs)
                grad_sink.done(W)
                return None, None, None, None, None, None
        return None, (Ct @ gs).float(), None, None, None, None


def embedding_bag(ids: torch.Tensor, W: torch.Tensor, W16: Optional[torch.Tensor] = None, pad: int = 0,
                  mean: bool = True, plan: str = "auto") -> torch.Tensor:
    """(N, L) ids -> (N, E): sum (or mean) of the rows of W over non-pad tokens."""
    if use_hip(ids, W):
        if W16 is None:
            W16 = W.detach().to(torch.bfloat16).contiguous()
        if plan == "auto":
            plan = "gather" if ids.shape[1] <= 256 else "counts"
        if W.shape[1] % 8:
            plan = "counts"
        return _BagFn.apply(ids, W, W16, pad, mean, plan)
    out = ref.embedding_bag_sum(ids, W, pad)
    if mean:
        out = out / (ids != pad).sum(dim=1, keepdim=True).clamp(min=1).to(out.dtype)
    return out


def trigram_hash(text: torch.Tensor, lens: torch.Tensor, L: int, hash_size: int) -> torch.Tensor:
    """Device letter-trigram hashing of ASCII byte rows (uint8 (N, Lmax)) -> int32 (N, L)."""
    if use_hip(text):
        N, Lmax = text.shape
        out = torch.empty(N, L, dtype=torch.int32, device=text.device)
        check(lib().pv_trigram_hash(P(text.contiguous()), P(lens.to(torch.int32).contiguous()), P(out), N, Lmax, L,
                                    hash_size, stream(text.device)), "pv_trigram_hash")
        return out
    return ref.fnv1a_trigram_ids(text.cpu(), lens.cpu(), L, hash_size).to(text.device)

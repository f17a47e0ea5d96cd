"""Blocked cosine top-k (K9).  GPU: HIP kernel (csrc/kernels/topk.hip); CPU: torch."""
from __future__ import annotations

from typing import Tuple

import torch

from ._common import P, check, lib, stream, use_hip


def _topk_torch(qn, pn, k, block):
    best_s = None
    best_i = None
    for s in range(0, pn.shape[0], block):
        sc = qn.float() @ pn[s:s + block].float().t()
        kk = min(k, sc.shape[1])
        v, i = sc.topk(kk, dim=1)
        i = i + s
        if best_s is None:
            best_s, best_i = v, i
        else:
            cs = torch.cat([best_s, v], 1)
            ci = torch.cat([best_i, i], 1)
            v2, j = cs.topk(min(k, cs.shape[1]), dim=1)
            best_s, best_i = v2, ci.gather(1, j)
    return best_s, best_i


def topk_cos(qn: torch.Tensor, pn: torch.Tensor, k: int = 10, block: int = 65536) -> Tuple[torch.Tensor, torch.Tensor]:
    if use_hip(qn, pn) and hasattr(lib(), "pv_topk_cos") and k <= 16 and qn.shape[1] <= 768:
        return _topk_hip(qn, pn, k)
    return _topk_torch(qn, pn, k, block)


_KS = (1, 2, 3, 4, 5, 6, 8, 12, 16, 24)
MAX_K = 16  # register-resident sorted lists of the kernel (topk.hip K)


def padded_width(D: int) -> int:
    """Zero-padded feature width: one of the kernel's compiled 32-multiples (topk.hip)."""
    return 32 * next(ks for ks in _KS if 32 * ks >= D)


def pad_bf16(x: torch.Tensor, DP: int) -> torch.Tensor:
    out = torch.zeros(x.shape[0], DP, dtype=torch.bfloat16, device=x.device)
    out[:, :x.shape[1]] = x
    return out


def topk_cos_padded(qb: torch.Tensor, pb: torch.Tensor, k: int, n: int = -1) -> Tuple[torch.Tensor, torch.Tensor]:
    """Top-k over the first ``n`` rows of PRE-PADDED bf16 pages ``pb`` (N_cap, DP) for
    pre-padded bf16 queries ``qb`` (B, DP) — the serving index keeps its pages in this
    layout so a search does not re-pad the collection.  k <= MAX_K; GPU only."""
    n = pb.shape[0] if n < 0 else n
    B, DP = qb.shape
    vals = torch.empty(B, k, dtype=torch.float32, device=qb.device)
    idx = torch.empty(B, k, dtype=torch.int32, device=qb.device)
    ns = int(lib().pv_topk_splits(B, n))
    pv = torch.full((B, ns, 4, 16), float("-inf"), dtype=torch.float32, device=qb.device)
    pi = torch.full((B, ns, 4, 16), -1, dtype=torch.int32, device=qb.device)
    check(lib().pv_topk_cos(P(qb), P(pb), P(vals), P(idx), P(pv), P(pi), B, n, DP, k, ns, stream(qb.device)),
          "pv_topk_cos")
    return vals, idx.long()


def _topk_hip(qn, pn, k):
    B, D = qn.shape
    N = pn.shape[0]
    DP = padded_width(D)
    qb = pad_bf16(qn, DP)
    pb = pad_bf16(pn, DP)
    vals = torch.empty(B, k, dtype=torch.float32, device=qn.device)
    idx = torch.empty(B, k, dtype=torch.int32, device=qn.device)
    ns = int(lib().pv_topk_splits(B, N))
    pv = torch.full((B, ns, 4, 16), float("-inf"), dtype=torch.float32, device=qn.device)
    pi = torch.full((B, ns, 4, 16), -1, dtype=torch.int32, device=qn.device)
    check(lib().pv_topk_cos(P(qb), P(pb), P(vals), P(idx), P(pv), P(pi), B, N, DP, k, ns, stream(qn.device)),
          "pv_topk_cos")
    return vals, idx.long()

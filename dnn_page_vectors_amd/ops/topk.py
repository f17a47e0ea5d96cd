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


def _topk_hip(qn, pn, k):
    B, D = qn.shape
    N = pn.shape[0]
    # zero-padded feature width: one of the kernel's compiled 32-multiples (topk.hip)
    DP = 32 * next(ks for ks in _KS if 32 * ks >= D)
    qb = torch.zeros(B, DP, dtype=torch.bfloat16, device=qn.device)
    qb[:, :D] = qn
    pb = torch.zeros(N, DP, dtype=torch.bfloat16, device=qn.device)
    pb[:, :D] = pn
    vals = torch.empty(B, k, dtype=torch.float32, device=qn.device)
    idx = torch.empty(B, k, dtype=torch.int32, device=qn.device)
    ns = int(lib().pv_topk_splits(B, N))
    pv = torch.full((B, ns, 4, 16), float("-inf"), dtype=torch.float32, device=qn.device)
    pi = torch.full((B, ns, 4, 16), -1, dtype=torch.int32, device=qn.device)
    check(lib().pv_topk_cos(P(qb), P(pb), P(vals), P(idx), P(pv), P(pi), B, N, DP, k, ns, stream(qn.device)),
          "pv_topk_cos")
    return vals, idx.long()

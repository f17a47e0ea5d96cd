"""Recall@k of queries against an encoded page collection (K9).

Brute-force cosine top-k: S = Qn . Pn^T in blocks, per-row top-k kept on device
(HIP kernel ``pv_topk_cos`` when available, torch.topk on CPU).  Recall@k is the
fraction of queries whose relevant page is among the k best-scoring pages — the
quality metric BASELINE.json adds (the reference only reported Keras accuracy,
dssm_cnn_v2/cnn_dssm_th.py:182).
"""
from __future__ import annotations

from typing import Dict, Sequence, Tuple

import torch
import torch.distributed as dist

from ..ops import topk as tops


def topk_cosine(qn: torch.Tensor, pn: torch.Tensor, k: int = 10, block: int = 65536) -> Tuple[torch.Tensor, torch.Tensor]:
    """(scores, indices) of the k most similar pages for every query (inputs normalised)."""
    return tops.topk_cos(qn, pn, k, block)


def recall_at_k(qn: torch.Tensor, pn: torch.Tensor, relevant: torch.Tensor, k: int = 10) -> float:
    """relevant[i] = index of query i's relevant page in ``pn``."""
    _, idx = topk_cosine(qn, pn, k)
    hit = (idx == relevant.view(-1, 1).to(idx.dtype)).any(dim=1)
    return float(hit.float().mean())


def recall_table(qn: torch.Tensor, pn: torch.Tensor, relevant: torch.Tensor, ks=(1, 10, 100)) -> dict:
    kmax = min(max(ks), pn.shape[0])
    _, idx = topk_cosine(qn, pn, kmax)
    rel = relevant.view(-1, 1).to(idx.dtype)
    return {f"recall@{k}": float((idx[:, :min(k, kmax)] == rel).any(dim=1).float().mean()) for k in ks}


def _gather_rows(x: torch.Tensor) -> Tuple[torch.Tensor, list]:
    """All-gather (n_r, D) row blocks of possibly different n_r from every rank, in rank
    order; returns (rows, [n_0, ..., n_{W-1}]).  RCCL gathers on the device, gloo on the host."""
    W = dist.get_world_size()
    comm = x.device if dist.get_backend() == "nccl" else torch.device("cpu")
    n = torch.tensor([x.shape[0]], dtype=torch.long, device=comm)
    ns = [torch.zeros_like(n) for _ in range(W)]
    dist.all_gather(ns, n)
    ns = [int(t) for t in ns]
    m = max(ns)
    buf = torch.zeros(m, x.shape[1], dtype=x.dtype, device=comm)
    buf[:x.shape[0]] = x.to(comm)
    parts = [torch.empty_like(buf) for _ in range(W)]
    dist.all_gather(parts, buf)
    rows = torch.cat([p[:k] for p, k in zip(parts, ns)], 0).to(x.device)
    return rows, ns


def distributed_recall_table(qn: torch.Tensor, pn: torch.Tensor, relevant: torch.Tensor,
                             ks: Sequence[int] = (1, 10, 100)) -> Dict[str, float]:
    """Recall@k over the pages of ALL ranks (all_gather(encoded pages) for the
    distributed Recall eval).

    Every rank holds its own queries ``qn`` (n_q, D), its own encoded pages ``pn`` (n_p, D)
    and ``relevant`` = the LOCAL page index of each query's relevant page.  The page vectors
    are all-gathered (rank order), each rank ranks its queries against the whole collection
    (relevant index shifted by the rank's page offset), and the hit counts are summed over
    ranks — the same numbers a single process would get with every rank's queries and pages
    concatenated in rank order.  Single process: ``recall_table``."""
    if not dist.is_initialized() or dist.get_world_size() == 1:
        return recall_table(qn, pn, relevant, ks)
    rank = dist.get_rank()
    allp, ns = _gather_rows(pn)
    offset = sum(ns[:rank])
    kmax = min(max(ks), allp.shape[0])
    _, idx = topk_cosine(qn, allp, kmax)
    rel = (relevant.view(-1, 1).to(idx.dtype) + offset)
    comm = qn.device if dist.get_backend() == "nccl" else torch.device("cpu")
    hits = torch.tensor([float((idx[:, :min(k, kmax)] == rel).any(dim=1).sum()) for k in ks] + [float(qn.shape[0])],
                        dtype=torch.float64, device=comm)
    dist.all_reduce(hits)
    total = float(hits[-1])
    return {f"recall@{k}": float(hits[i]) / max(1.0, total) for i, k in enumerate(ks)}

"""Recall@k of queries against an encoded page collection (K9).

Brute-force cosine top-k: S = Qn . Pn^T in blocks, per-row top-k kept on device
(HIP kernel ``pv_topk_cos`` when available, torch.topk on CPU).  Recall@k is the
fraction of queries whose relevant page is among the k best-scoring pages — the
quality metric BASELINE.json adds (the reference only reported Keras accuracy,
dssm_cnn_v2/cnn_dssm_th.py:182).
"""
from __future__ import annotations

from typing import Tuple

import torch

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

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
from ..parallel.dist import active as pdist_active


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
    if not pdist_active():
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


def _hits(qn: torch.Tensor, pages: torch.Tensor, relevant: torch.Tensor, ks: Sequence[int]) -> list:
    kmax = min(max(ks), pages.shape[0])
    _, idx = topk_cosine(qn, pages, kmax)
    rel = relevant.view(-1, 1).to(idx.dtype)
    return [float((idx[:, :min(k, kmax)] == rel).any(dim=1).sum()) for k in ks]


@torch.no_grad()
def evaluate_pairs_dataset(model, dataset, device: torch.device, ks: Sequence[int] = (1, 10, 100),
                           max_rows: int = 0, include_negatives: bool = True, batch: int = 1024) -> Dict[str, float]:
    """Recall@k on a real {'q', 'doc_corr', 'doc_incorr'} JSONL file (``data.dataset.JsonlPairDataset``):
    the reference's per-epoch validation pass over ``model_validation_data``
    (dssm_cnn_v2/cnn_dssm_th.py:189-194), measured as retrieval instead of Keras accuracy.

    Every row's query is ranked against the collection of all distinct pages of the file
    (the positives, plus the rows' negatives as distractors when ``include_negatives``);
    a query hits when its own positive page is in the top k.  Pages are de-duplicated by
    their featurized ids (the same page text in several rows is ONE page).

    Under a process group (collective: every rank calls it) every rank featurizes the rows
    (host work) so all ranks agree on the distinct-page numbering, encodes its contiguous
    shard of the queries and of the distinct pages, all-gathers the page vectors
     and the hit counts are summed: the result equals the single-process one."""
    distributed = pdist_active()
    rank, W = (dist.get_rank(), dist.get_world_size()) if distributed else (0, 1)
    n = len(dataset)
    if max_rows:
        n = min(n, int(max_rows))
    if n == 0:
        raise ValueError("no rows to evaluate")
    qs, pages, rel, index = [], [], [], {}

    def page_id(ids_row) -> int:
        key = ids_row.tobytes()
        j = index.get(key)
        if j is None:
            j = index[key] = len(pages)
            pages.append(ids_row.copy())
        return j

    import numpy as np

    for s in range(0, n, batch):
        q, d = dataset.batch(np.arange(s, min(n, s + batch)))
        for i in range(q.shape[0]):
            rel.append(page_id(d[i, 0]))
            if include_negatives:
                for j in range(1, d.shape[1]):
                    page_id(d[i, j])
        qs.append(q)
    q_all = np.concatenate(qs)
    P = len(pages)

    def shard(m: int):
        per = -(-m // W)
        return min(m, rank * per), min(m, (rank + 1) * per)

    q0, q1 = shard(n)
    p0, p1 = shard(P)
    enc_q = model.encode(torch.from_numpy(q_all[q0:q1]).to(device), "query", batch_size=batch) if q1 > q0 else None
    p_local = torch.from_numpy(np.stack(pages[p0:p1])).to(device) if p1 > p0 else None
    pv = model.encode(p_local, "doc", batch_size=batch) if p_local is not None else None
    D = model.out_dim
    if pv is None:
        pv = torch.empty(0, D, device=device)
    allp = _gather_rows(pv.float())[0] if distributed else pv
    relevant = torch.tensor(rel[q0:q1], device=device)
    hits = _hits(enc_q, allp, relevant, ks) if enc_q is not None else [0.0] * len(ks)
    comm = device if (distributed and dist.get_backend() == "nccl") else torch.device("cpu")
    h = torch.tensor(hits + [float(q1 - q0)], dtype=torch.float64, device=comm)
    if distributed:
        dist.all_reduce(h)
    out = {f"recall@{k}": float(h[i]) / max(1.0, float(h[-1])) for i, k in enumerate(ks)}
    out["queries"] = int(n)
    out["pages"] = int(P)
    return out

"""Page-vector index: the serving side of ``encode()``.

The reference stops at training (its only "extract vectors" pattern is reading a weight
matrix, old_scripts/simple_rnn.py:51); a production deployment encodes the page
collection once and answers queries by cosine top-k.  ``PageIndex`` keeps the
L2-normalised page vectors resident in HBM in the exact layout the HIP top-k kernel
reads (zero-padded bf16 rows, ``ops/topk.py::topk_cos_padded``), grows by doubling, and
maps row numbers to caller ids.  A 288 GB MI355X holds ~900 M 150-d pages per GPU in
this layout; ``ShardedPageIndex`` spreads a larger collection over the ranks of a
process group (each rank searches its shard, one all-gather of the (k scores, k ids)
per query batch, merged on every rank).

CPU: the same API over fp32 tensors and ``torch.topk`` (tests, small collections).
Persistence: ``save(path)`` writes ``<path>.safetensors`` (vectors) + ``<path>.json``
(ids, dimension) — no pickles.
"""
from __future__ import annotations

import json
import os
from typing import List, Optional, Sequence, Tuple, Union

import torch
import torch.distributed as dist

from ..ops import topk as tops

IdT = Union[int, str]


class PageIndex:
    def __init__(self, dim: int, device: Optional[Union[str, torch.device]] = None, capacity: int = 1024):
        self.dim = int(dim)
        self.device = torch.device(device) if device is not None else (
            torch.device("cuda") if torch.cuda.is_available() else torch.device("cpu"))
        self.gpu = self.device.type == "cuda"
        self.DP = tops.padded_width(self.dim) if self.gpu else self.dim
        self.n = 0
        self.ids: List[IdT] = []
        self._rows = torch.zeros(max(1, capacity), self.DP, dtype=torch.bfloat16 if self.gpu else torch.float32,
                                 device=self.device)

    def __len__(self) -> int:
        return self.n

    @property
    def capacity(self) -> int:
        return self._rows.shape[0]

    def _reserve(self, n: int) -> None:
        if n <= self.capacity:
            return
        cap = self.capacity
        while cap < n:
            cap *= 2
        rows = torch.zeros(cap, self.DP, dtype=self._rows.dtype, device=self.device)
        rows[:self.n] = self._rows[:self.n]
        self._rows = rows

    @torch.no_grad()
    def add(self, vectors: torch.Tensor, ids: Optional[Sequence[IdT]] = None, normalize: bool = True) -> None:
        """Append page vectors (N, dim); ids default to consecutive row numbers."""
        if vectors.dim() != 2 or vectors.shape[1] != self.dim:
            raise ValueError(f"expected (N, {self.dim}) vectors, got {tuple(vectors.shape)}")
        m = vectors.shape[0]
        if ids is None:
            ids = list(range(self.n, self.n + m))
        if len(ids) != m:
            raise ValueError("one id per vector")
        v = vectors.to(self.device, torch.float32)
        if normalize:
            v = v / v.norm(dim=1, keepdim=True).clamp_min(1e-12)
        self._reserve(self.n + m)
        self._rows[self.n:self.n + m, :self.dim] = v.to(self._rows.dtype)
        self.n += m
        self.ids.extend(ids)

    @torch.no_grad()
    def search_rows(self, queries: torch.Tensor, k: int = 10, normalize: bool = True
                    ) -> Tuple[torch.Tensor, torch.Tensor]:
        """(scores (B, k'), row numbers (B, k')) with k' = min(k, len(self)); rows -1 pad."""
        if queries.dim() != 2 or queries.shape[1] != self.dim:
            raise ValueError(f"expected (B, {self.dim}) queries")
        B = queries.shape[0]
        kk = min(int(k), self.n)
        if kk == 0 or B == 0:
            return (torch.empty(B, 0, device=self.device), torch.empty(B, 0, dtype=torch.long, device=self.device))
        q = queries.to(self.device, torch.float32)
        if normalize:
            q = q / q.norm(dim=1, keepdim=True).clamp_min(1e-12)
        if self.gpu and kk <= tops.MAX_K:
            return tops.topk_cos_padded(tops.pad_bf16(q, self.DP), self._rows, kk, self.n)
        pages = self._rows[:self.n, :self.dim].float()
        best_v, best_i = None, None
        for s in range(0, self.n, 1 << 18):  # bounded (B x block) score tiles
            sc = q @ pages[s:s + (1 << 18)].t()
            v, i = sc.topk(min(kk, sc.shape[1]), dim=1)
            i = i + s
            if best_v is None:
                best_v, best_i = v, i
            else:
                cv, ci = torch.cat([best_v, v], 1), torch.cat([best_i, i], 1)
                best_v, j = cv.topk(kk, dim=1)
                best_i = ci.gather(1, j)
        return best_v, best_i

    def search(self, queries: torch.Tensor, k: int = 10) -> List[List[Tuple[IdT, float]]]:
        """Per query, [(id, cosine score)] best first."""
        v, i = self.search_rows(queries, k)
        v, i = v.cpu().tolist(), i.cpu().tolist()
        return [[(self.ids[r], s) for r, s in zip(ri, vi) if r >= 0] for ri, vi in zip(i, v)]

    def vectors(self) -> torch.Tensor:
        return self._rows[:self.n, :self.dim].float()

    def save(self, path: str) -> None:
        from safetensors.torch import save_file

        os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
        save_file({"vectors": self.vectors().cpu().contiguous()}, path + ".safetensors")
        with open(path + ".json", "w", encoding="utf-8") as f:
            json.dump({"dim": self.dim, "ids": self.ids}, f)

    @classmethod
    def load(cls, path: str, device: Optional[Union[str, torch.device]] = None) -> "PageIndex":
        from safetensors.torch import load_file

        with open(path + ".json", encoding="utf-8") as f:
            meta = json.load(f)
        vec = load_file(path + ".safetensors")["vectors"]
        idx = cls(meta["dim"], device=device, capacity=max(1, vec.shape[0]))
        idx.add(vec, meta["ids"], normalize=False)
        return idx


class ShardedPageIndex:
    """A page collection split over the ranks of a process group: rank r owns the pages
    added on it; ``search`` runs the local top-k on every rank, all-gathers the (B, k)
    candidate lists and merges them — the result is identical on every rank.  Every
    rank must call ``search`` with the same queries (collective)."""

    def __init__(self, local: PageIndex, group=None):
        self.local = local
        self.group = group

    def __len__(self) -> int:
        n = torch.tensor([len(self.local)], dtype=torch.long, device=self._comm_device())
        if dist.is_initialized():
            dist.all_reduce(n, group=self.group)
        return int(n)

    def _comm_device(self) -> torch.device:
        if dist.is_initialized() and dist.get_backend(self.group) == "nccl":
            return self.local.device
        return torch.device("cpu")

    def search(self, queries: torch.Tensor, k: int = 10) -> List[List[Tuple[IdT, float]]]:
        if not dist.is_initialized() or dist.get_world_size(self.group) == 1:
            return self.local.search(queries, k)
        W = dist.get_world_size(self.group)
        B = queries.shape[0]
        v, r = self.local.search_rows(queries, k)
        kk = int(k)
        # pad to k columns: (-inf, -1) where the shard has fewer pages
        pv = torch.full((B, kk), float("-inf"), dtype=torch.float32, device=v.device)
        pr = torch.full((B, kk), -1, dtype=torch.long, device=v.device)
        pv[:, :v.shape[1]] = v.float()
        pr[:, :r.shape[1]] = r
        dev = self._comm_device()
        allv = [torch.empty(B, kk, dtype=torch.float32, device=dev) for _ in range(W)]
        dist.all_gather(allv, pv.to(dev), group=self.group)
        # ids live on their owning rank: every rank contributes the ids of its B x k candidates
        ids_all: List[List[IdT]] = [None] * W  # type: ignore[list-item]
        dist.all_gather_object(ids_all, [self.local.ids[int(x)] if x >= 0 else None for x in pr.reshape(-1).tolist()],
                               group=self.group)
        cv = torch.cat(allv, 1)                       # (B, W*k)
        owner = torch.arange(W).repeat_interleave(kk).unsqueeze(0).expand(B, -1)
        col = torch.arange(kk).repeat(W).unsqueeze(0).expand(B, -1)
        best, j = cv.cpu().topk(min(kk, cv.shape[1]), dim=1)
        out = []
        for b in range(B):
            row = []
            for s, jj in zip(best[b].tolist(), j[b].tolist()):
                w, c = int(owner[b, jj]), int(col[b, jj])
                pid = ids_all[w][b * kk + c]
                if pid is not None and s != float("-inf"):
                    row.append((pid, s))
            out.append(row)
        return out


__all__ = ["PageIndex", "ShardedPageIndex"]

"""Synthetic query/page pairs (no dataset download is possible on the GPU box).

Pages are topical token-id sequences (ids in [1, V), 0 = PAD): each position draws,
with probability ``topic_frac``, from the page's own small topic vocabulary and
otherwise from a global Zipf background (the common words every page shares).  The
query of a page is a noisy contiguous sub-span of it (10% of its tokens replaced by
random background tokens), so relevance is learnable and Recall@10 is a meaningful
quality signal.
Negatives are other random pages (the reference's J=3 explicit negatives,
dssm_cnn_v2/data_helpers.py:163-192).

Everything is generated with torch on the target device from a fixed seed, so a
benchmark can keep an HBM-resident page pool and gather its batches on device.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional, Tuple

import torch


@dataclass
class SyntheticSpec:
    vocab_size: int
    query_length: int
    document_length: int
    num_negatives: int = 3
    num_pages: int = 65536
    zipf_s: float = 1.05
    query_noise: float = 0.1
    min_query_frac: float = 0.34
    var_doc_len: bool = False
    topic_frac: float = 0.5      # share of a page's tokens drawn from its own topic vocabulary
    topic_size: int = 32         # distinct topic tokens per page


class SyntheticPairs:
    def __init__(self, spec: SyntheticSpec, device: torch.device | str = "cpu", seed: int = 1337,
                 vocab_seed: int = 1337):
        """``seed`` draws the pages / queries / batches (data-parallel ranks pass rank-specific
        seeds); ``vocab_seed`` fixes the token-frequency "language" (which id is the k-th most
        frequent token), shared by every rank so all ranks train on one distribution."""
        self.spec = spec
        self.device = torch.device(device)
        self.gen = torch.Generator(device="cpu").manual_seed(seed)
        V = spec.vocab_size
        ranks = torch.arange(1, V, dtype=torch.float64)
        probs = ranks.pow(-spec.zipf_s)
        # random permutation of ids so frequent tokens are spread over the id space (as hashing does)
        perm = torch.randperm(V - 1, generator=torch.Generator(device="cpu").manual_seed(vocab_seed)) + 1
        self.cdf = torch.cumsum(probs / probs.sum(), 0).float().to(self.device)
        self.id_of_rank = perm.to(torch.int32).to(self.device)
        self.pages = self._sample_pages(spec.num_pages)
        if spec.var_doc_len:
            lens = torch.randint(spec.document_length // 2, spec.document_length + 1, (spec.num_pages,),
                                 generator=self.gen).to(self.device)
            pos = torch.arange(spec.document_length, device=self.device)
            self.pages[pos[None, :] >= lens[:, None]] = 0

    def _rand(self, *shape) -> torch.Tensor:
        return torch.rand(*shape, generator=self.gen).to(self.device)

    def _sample_tokens(self, n: int, L: int) -> torch.Tensor:
        out = torch.empty(n, L, dtype=torch.int32, device=self.device)
        chunk = max(1, (1 << 24) // max(1, L))
        for i in range(0, n, chunk):
            m = min(chunk, n - i)
            u = self._rand(m, L)
            r = torch.searchsorted(self.cdf, u.reshape(-1)).clamp_(max=self.cdf.numel() - 1)
            out[i:i + m] = self.id_of_rank[r].view(m, L)
        return out

    def _sample_pages(self, n: int) -> torch.Tensor:
        s = self.spec
        L = s.document_length
        pages = self._sample_tokens(n, L)
        if s.topic_frac > 0 and s.topic_size > 0:
            chunk = max(1, (1 << 24) // max(1, L))
            for i in range(0, n, chunk):
                m = min(chunk, n - i)
                topics = (1 + (self._rand(m, s.topic_size) * (s.vocab_size - 1)).long()).clamp_(max=s.vocab_size - 1)
                pick = (self._rand(m, L) * s.topic_size).long().clamp_(max=s.topic_size - 1)
                tok = torch.gather(topics, 1, pick).to(torch.int32)
                use = self._rand(m, L) < s.topic_frac
                pages[i:i + m] = torch.where(use, tok, pages[i:i + m])
        return pages

    def queries_for(self, page_idx: torch.Tensor) -> torch.Tensor:
        """Noisy sub-span queries (n, Lq) for the given page indices."""
        s = self.spec
        n = page_idx.numel()
        Lq, Ld = s.query_length, s.document_length
        lo = max(3, int(Lq * s.min_query_frac))
        qlen = (lo + (self._rand(n) * (Lq - lo + 1)).long()).clamp_(max=Lq)
        start = (self._rand(n) * (Ld - qlen + 1).float()).long()
        pos = torch.arange(Lq, device=self.device)
        src = (start[:, None] + pos[None, :]).clamp_(max=Ld - 1)
        q = torch.gather(self.pages[page_idx.long()], 1, src)
        noise = self._rand(n, Lq) < s.query_noise
        q = torch.where(noise, self._sample_tokens(n, Lq), q)
        q[pos[None, :] >= qlen[:, None]] = 0
        return q.to(torch.int32)

    def batch(self, batch_size: int) -> Tuple[torch.Tensor, torch.Tensor]:
        """(q_ids (B, Lq), d_ids (B, 1+J, Ld)) with the positive page first."""
        J = self.spec.num_negatives
        P = self.spec.num_pages
        idx = (self._rand(batch_size) * P).long().clamp_(max=P - 1)
        q = self.queries_for(idx)
        if J > 0:
            neg = (idx[:, None] + 1 + (self._rand(batch_size, J) * (P - 1)).long()) % P
            didx = torch.cat([idx[:, None], neg], dim=1)
        else:
            didx = idx[:, None]
        d = self.pages[didx]
        return q, d

    def eval_set(self, num_pages: int, seed: int = 7) -> Tuple[torch.Tensor, torch.Tensor]:
        """Held-out (queries, pages) where query i's relevant page is page i."""
        g = self.gen
        self.gen = torch.Generator(device="cpu").manual_seed(seed)
        try:
            pages = self._sample_pages(num_pages)
            saved = self.pages
            self.pages = pages
            q = self.queries_for(torch.arange(num_pages, device=self.device))
            self.pages = saved
        finally:
            self.gen = g
        return q, pages


def spec_from_config(cfg, vocab_size: Optional[int] = None, num_pages: int = 65536) -> SyntheticSpec:
    V = vocab_size or (cfg.vocab_hash_size if cfg.vocab_hash_size > 1 else 1000)
    return SyntheticSpec(vocab_size=V, query_length=cfg.query_length, document_length=cfg.document_length,
                         num_negatives=cfg.J, num_pages=num_pages)

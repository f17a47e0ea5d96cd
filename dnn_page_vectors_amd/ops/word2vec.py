"""Word2Vec SGD over a chunk of center positions (negative sampling, CBOW or skip-gram).

GPU: ``csrc/kernels/w2v.hip`` (one wave per center, atomic-add updates).  CPU / oracle:
``train_chunk_torch`` — the same algorithm in plain fp32 torch, vectorised over the
centers of a mini-batch and sequential over the targets of a center, so with
``batch=1`` it reproduces the kernel's arithmetic order for one center exactly (the
counter RNG below is the kernel's ``w2v_rng``).

Reference: gensim's training loop as called by ``train_word2vec``
(dssm_cnn_v2/w2v.py:37-39; gensim word2vec_inner ``fast_sentence_cbow_neg`` /
``fast_sentence_sg_neg``).  Differences: the logistic uses the exact sigmoid instead of
gensim's 1000-entry EXP_TABLE with MAX_EXP = 6 clipping.
"""
from __future__ import annotations

import torch

from ._common import P, check, lib, stream, use_hip
from .reference import _M32, _mix32

_GOLDEN = 0x9E3779B9


def w2v_rng(seed: int, i: torch.Tensor, k) -> torch.Tensor:
    """mix32(mix32(seed ^ i) + k * golden) on int64 tensors holding uint32 values."""
    a = _mix32((i & _M32) ^ (int(seed) & _M32))
    if isinstance(k, torch.Tensor):
        kk = (k * _GOLDEN) & _M32
    else:
        kk = (int(k) * _GOLDEN) & _M32
    return _mix32((a + kk) & _M32)


def train_chunk(words: torch.Tensor, sbeg: torch.Tensor, send: torch.Tensor, table: torch.Tensor,
                win: torch.Tensor, wout: torch.Tensor, begin: int, end: int, window: int, negative: int,
                seed: int, alpha: float, sg: bool, batch: int = 1024) -> None:
    """Train centers [begin, end) in place (int32 corpus / bounds / table, fp32 tables)."""
    if end <= begin:
        return
    if use_hip(win, wout):
        D = win.shape[1]
        check(lib().pv_w2v_train(P(words), P(sbeg), P(send), P(table), P(win), P(wout), int(begin), int(end),
                                 table.numel(), D, int(window), int(negative), int(seed) & _M32, float(alpha),
                                 int(bool(sg)), stream(win.device)), "pv_w2v_train")
        return
    for b0 in range(begin, end, batch):
        train_chunk_torch(words, sbeg, send, table, win, wout, b0, min(end, b0 + batch), window, negative, seed,
                          alpha, sg)


@torch.no_grad()
def _targets_step(win_h: torch.Tensor, e: torch.Tensor, wout: torch.Tensor, table: torch.Tensor, ctr: torch.Tensor,
                  kbase: torch.Tensor, center: torch.Tensor, live: torch.Tensor, negative: int, seed: int,
                  alpha: float) -> None:
    """Positive + negatives for a batch of (h, center) pairs; updates wout, accumulates e."""
    for k in range(negative + 1):
        if k == 0:
            t = center
            label = 1.0
            ok = live
        else:
            r = w2v_rng(seed, ctr, kbase + k)
            t = table[(r % table.numel()).long()].long()
            label = 0.0
            ok = live & (t != center)
        o = wout[t]
        f = (win_h * o).sum(-1)
        g = (label - torch.sigmoid(f)) * alpha * ok.float()
        e += g[:, None] * o
        wout.index_add_(0, t, g[:, None] * win_h)


@torch.no_grad()
def train_chunk_torch(words, sbeg, send, table, win, wout, begin, end, window, negative, seed, alpha, sg) -> None:
    dev = win.device
    i = torch.arange(begin, end, device=dev, dtype=torch.int64)
    ctr = i & _M32
    w = window - (w2v_rng(seed, ctr, 0) % window)
    lo = torch.maximum(sbeg[i].long(), i - w)
    hi = torch.minimum(send[i].long(), i + w + 1)
    center = words[i].long()
    T = words.numel()
    offs = [o for o in range(-window, window + 1) if o != 0]
    if not sg:
        h = torch.zeros(i.numel(), win.shape[1], device=dev, dtype=win.dtype)
        cnt = torch.zeros(i.numel(), device=dev, dtype=win.dtype)
        ctx = []
        for o in offs:
            c = i + o
            valid = (c >= lo) & (c < hi)
            cw = words[c.clamp(0, T - 1)].long()
            h += win[cw] * valid[:, None].float()
            cnt += valid.float()
            ctx.append((cw, valid))
        live = cnt > 0
        h = h / cnt.clamp(min=1.0)[:, None]
        e = torch.zeros_like(h)
        _targets_step(h, e, wout, table, ctr, torch.zeros_like(ctr), center, live, negative, seed, alpha)
        for cw, valid in ctx:
            win.index_add_(0, cw, e * valid[:, None].float())
    else:
        for o in offs:  # increasing context index c = i + o, as the kernel's loop
            c = i + o
            valid = (c >= lo) & (c < hi)
            cw = words[c.clamp(0, T - 1)].long()
            h = win[cw]
            e = torch.zeros_like(h)
            kbase = ((c - lo).clamp(min=0) * negative) & _M32
            _targets_step(h, e, wout, table, ctr, kbase, center, valid, negative, seed, alpha)
            win.index_add_(0, cw, e * valid[:, None].float())

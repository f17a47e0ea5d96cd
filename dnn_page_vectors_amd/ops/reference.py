"""Plain-PyTorch (fp32) reference implementations of every hot op.

These are (1) the numerics oracle the HIP kernels are tested against and
(2) the CPU execution path (tests, config 1).  They are written for clarity,
not speed.  Semantics follow the reference model graph
``dssm_cnn_v2/cnn_dssm_th.py:63-182``.

Dropout masks are counter-based (a pure function of ``(seed, row, column)``)
so the fused HIP forward and the sparse backward regenerate the identical
mask without storing it; ``dropout_keep_mask`` defines that function.
"""
from __future__ import annotations

import math
from typing import List, Optional, Sequence, Tuple

import numpy as np
import torch
import torch.nn.functional as F

FLT_TINY = float(np.finfo(np.float32).tiny)  # np.finfo(x.dtype).tiny, cnn_dssm_th.py:70-74
BCE_EPS = 1e-7                                 # Keras epsilon() clip in binary_crossentropy

_M32 = 0xFFFFFFFF


def _mix32(x: torch.Tensor) -> torch.Tensor:
    """lowbias32 finaliser on int64 tensors holding uint32 values."""
    x = x & _M32
    x = x ^ (x >> 16)
    x = (x * 0x7FEB352D) & _M32
    x = x ^ (x >> 15)
    x = (x * 0x846CA68B) & _M32
    x = x ^ (x >> 16)
    return x


_GROUP_STEP = 0x9E3779  # 24-bit golden-ratio step between a row's groups
# nibble mode: element j of a group reads h[P] h[P-8] h[P-4] h[P-12] (MSB first), P = 15 - j//2 + 16 (j%2)
_NIB_POS = [15 - (j >> 1) + 16 * (j & 1) for j in range(8)]


def _mix24(x: torch.Tensor) -> torch.Tensor:
    """The group-hash mixer (common.h mix24): two xorshift + 24-bit-multiply rounds."""
    x = x & _M32
    x = x ^ (x >> 16)
    x = ((x & 0xFFFFFF) * 0xED5AD5) & _M32
    x = x ^ (x >> 15)
    return ((x & 0xFFFFFF) * 0x9E3779) & _M32


def _group_hash(h_row: torch.Tensor, g: torch.Tensor) -> torch.Tensor:
    """(n,) row hashes x (ng,) group ids -> (n, ng) group hashes (common.h dropout_group_hash)."""
    return _mix24(h_row.unsqueeze(1) + ((g & 0xFFFFFF) * _GROUP_STEP).unsqueeze(0))


def dropout_threshold(p: float) -> int:
    """Keep an element when its 8-bit hash byte >= round(p*256) (p quantised to 1/256)."""
    return int(round(p * 256.0))


def dropout_keep_mask(seed: int, n_rows: int, width: int, p: float, row_offset: int = 0,
                      mode: str = "element", device=None, rows: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Bool keep-mask of shape (n_rows, width) for flat row ids ``row_offset + r`` (r < n_rows,
    or r in ``rows`` when given: any local row ids, n_rows = rows.numel()).

    h_row = mix32(row ^ mix32(seed)) (lowbias32); the group hash of group g of a row is
    h = mix24(h_row + g * 0x9E3779) (two xorshift / 24-bit multiply rounds, full-rate on the GPU).

    element, thr = round(256p) a multiple of 16 (p = k/16, e.g. the reference's 0.25): column
             8g + j is kept iff the 4-bit value h[P] h[P-8] h[P-4] h[P-12] (MSB first),
             P = 15 - j//2 + 16 (j%2), is >= thr/16 — one hash per 8 columns (the layout lets
             the kernels build the bf16 pair masks with v_perm_b32, common.h keep_piece);
    element, other thr: byte b of the group hash of g decides column 4g+b (>= thr);
    token:   one decision per row: byte 0 of h_row.
    """
    thr = dropout_threshold(p)
    if rows is None:
        rows = torch.arange(n_rows, dtype=torch.int64, device=device) + int(row_offset)
    else:
        rows = rows.reshape(-1).to(torch.int64) + int(row_offset)
        n_rows, device = rows.numel(), rows.device
    h_row = _mix32(rows ^ _mix32(torch.tensor(int(seed) & _M32, dtype=torch.int64, device=device)))
    if mode == "token":
        b = h_row & 0xFF
        return (b >= thr).unsqueeze(1).expand(n_rows, width)
    if thr % 16 == 0:
        ng = (width + 7) // 8
        g = torch.arange(ng, dtype=torch.int64, device=device)
        h = _group_hash(h_row, g).unsqueeze(2)  # (n, ng, 1)
        P = torch.tensor(_NIB_POS, dtype=torch.int64, device=device)
        nib = (((h >> P) & 1) << 3) | (((h >> (P - 8)) & 1) << 2) | (((h >> (P - 4)) & 1) << 1) | ((h >> (P - 12)) & 1)
        return nib.reshape(n_rows, ng * 8)[:, :width] >= thr // 16
    ng = (width + 3) // 4
    g = torch.arange(ng, dtype=torch.int64, device=device)
    h = _group_hash(h_row, g)  # (n, ng)
    shifts = torch.tensor([0, 8, 16, 24], dtype=torch.int64, device=device)
    bytes_ = (h.unsqueeze(2) >> shifts) & 0xFF  # (n, ng, 4)
    return (bytes_.reshape(n_rows, ng * 4)[:, :width] >= thr)


def embed_dropout(ids: torch.Tensor, table: torch.Tensor, p: float, seed: int, training: bool,
                  mode: str = "element") -> torch.Tensor:
    """Embedding gather (+ counter-based dropout, scale 1/(1-p)). ids (N, L) -> (N, L, E)."""
    x = F.embedding(ids.long(), table)
    if training and p > 0.0 and mode != "none":
        N, L, E = x.shape
        keep = dropout_keep_mask(seed, N * L, E, p, mode=mode, device=ids.device).view(N, L, E)
        scale = 256.0 / (256.0 - dropout_threshold(p))
        x = x * keep.to(x.dtype) * scale
    return x


def conv_relu_maxpool(x: torch.Tensor, weights: Sequence[torch.Tensor], biases: Sequence[torch.Tensor]
                      ) -> Tuple[torch.Tensor, torch.Tensor]:
    """Valid 1-D convs + ReLU + global max-pool over time + concat.

    x: (N, L, E); weights[i]: (F, k_i, E); biases[i]: (F,).
    Returns pooled (N, sum F) and argmax window positions (N, sum F) int32.
    """
    outs, args = [], []
    xt = x.transpose(1, 2)  # (N, E, L)
    for w, b in zip(weights, biases):
        k = w.shape[1]
        if x.shape[1] < k:
            raise ValueError(f"sequence length {x.shape[1]} shorter than filter width {k}")
        y = F.conv1d(xt, w.permute(0, 2, 1), b)  # (N, F, L-k+1)
        m, a = y.max(dim=2)
        outs.append(torch.relu(m))
        args.append(a.to(torch.int32))
    return torch.cat(outs, dim=1), torch.cat(args, dim=1)


def conv_maxpool_grads_at(x: torch.Tensor, weights: Sequence[torch.Tensor], pooled: torch.Tensor,
                          argmax: torch.Tensor, gpool: torch.Tensor):
    """fp32 backward of ``conv_relu_maxpool`` through GIVEN argmax windows (e.g. the fused
    kernel's own, so near-ties in the forward cannot make the comparison skip): with
    g = gpool * [pooled > 0],  dW[f, j] = sum_n g[n, f] x[n, a + j],  db[f] = sum_n g[n, f],
    dx[n, a + j] += g[n, f] W[f, j].  Returns ([dW_i], [db_i], dx)."""
    N, L, E = x.shape
    g = gpool * (pooled > 0).to(gpool.dtype)
    dx = torch.zeros_like(x)
    dws, dbs = [], []
    c = 0
    for w in weights:
        Fk, k, _ = w.shape
        gi = g[:, c:c + Fk]
        a = argmax[:, c:c + Fk].long()
        pos = a.unsqueeze(2) + torch.arange(k, device=x.device)           # (N, F, k)
        win = x[torch.arange(N, device=x.device)[:, None, None], pos]     # (N, F, k, E)
        dws.append(torch.einsum("nf,nfke->fke", gi, win))
        dbs.append(gi.sum(0))
        contrib = gi[:, :, None, None] * w.unsqueeze(0)                   # (N, F, k, E)
        dx.index_put_((torch.arange(N, device=x.device)[:, None, None].expand_as(pos), pos), contrib,
                      accumulate=True)
        c += Fk
    return dws, dbs, dx


def cdssm_tower_features(ids, table, weights, biases, p, seed, training, mode="element"):
    x = embed_dropout(ids, table, p, seed, training, mode)
    pooled, _ = conv_relu_maxpool(x, weights, biases)
    return pooled


def linear_act(x: torch.Tensor, w: torch.Tensor, b: Optional[torch.Tensor], act: str = "relu") -> torch.Tensor:
    """y = act(x @ w.T + b); w: (out, in)."""
    y = F.linear(x, w, b)
    if act == "relu":
        return torch.relu(y)
    if act == "gelu":
        return F.gelu(y, approximate="tanh")
    if act == "tanh":
        return torch.tanh(y)
    if act == "none":
        return y
    raise ValueError(act)


def l2_normalize(x: torch.Tensor) -> torch.Tensor:
    """x / sqrt(max(|x|^2, tiny)) — the RTH/RTF magnitude (cnn_dssm_th.py:66-75)."""
    sq = (x * x).sum(dim=-1, keepdim=True)
    return x / torch.sqrt(torch.clamp(sq, min=FLT_TINY))


def cosine_clip(q: torch.Tensor, d: torch.Tensor) -> torch.Tensor:
    """R(Q,D) = clip(q.d / (|q||d|), 0, 1) with the tiny-clamped squared norms."""
    return torch.clamp((l2_normalize(q) * l2_normalize(d)).sum(-1), 0.0, 1.0)


def dssm_explicit_loss(q: torch.Tensor, docs: torch.Tensor, gamma: float
                       ) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    """Reference-parity head: q (B, D), docs (B, 1+J, D) with the positive first.

    P = exp(gR+)/sum_j exp(gR_j); loss = mean(-log clip(P, 1e-7, 1-1e-7)) (Keras BCE, y=1).
    Returns (loss, P, R).
    """
    R = cosine_clip(q.unsqueeze(1), docs)          # (B, 1+J)
    e = torch.exp(gamma * R)
    P = e[:, 0] / e.sum(dim=1)
    loss = -torch.log(torch.clamp(P, BCE_EPS, 1.0 - BCE_EPS)).mean()
    return loss, P, R


def inbatch_softmax_loss(qn: torch.Tensor, dn: torch.Tensor, pos_index: torch.Tensor, gamma: float,
                         clip: bool = True) -> Tuple[torch.Tensor, torch.Tensor]:
    """In-batch / cross-GPU head on L2-normalised vectors.

    qn (B, D), dn (M, D): every query is scored against all M documents;
    ``pos_index[i]`` is the row of its positive. loss_i = -log softmax(g*R_i)[pos_i].
    Returns (per-row loss (B,), P_pos (B,)).
    """
    R = qn @ dn.t()
    if clip:
        R = torch.clamp(R, 0.0, 1.0)
    S = gamma * R
    lse = torch.logsumexp(S, dim=1)
    spos = S.gather(1, pos_index.long().view(-1, 1)).squeeze(1)
    loss = lse - spos
    return loss, torch.exp(-loss)


def embedding_bag_sum(ids: torch.Tensor, table: torch.Tensor, pad_id: int = 0) -> torch.Tensor:
    """Sum of embedding rows over non-pad ids: (N, L) -> (N, E) (multi-hot x W1 of DSSM)."""
    x = F.embedding(ids.long(), table)
    mask = (ids != pad_id).to(x.dtype).unsqueeze(-1)
    return (x * mask).sum(dim=1)


def adam_keras_(params: List[torch.Tensor], grads: List[torch.Tensor], ms: List[torch.Tensor],
                vs: List[torch.Tensor], step: int, lr: float, b1: float, b2: float, eps: float) -> None:
    """Keras-1 Adam: lr_t = lr*sqrt(1-b2^t)/(1-b1^t); p -= lr_t*m/(sqrt(v)+eps)."""
    lr_t = lr * math.sqrt(1.0 - b2 ** step) / (1.0 - b1 ** step)
    with torch.no_grad():
        for p, g, m, v in zip(params, grads, ms, vs):
            m.mul_(b1).add_(g, alpha=1 - b1)
            v.mul_(b2).addcmul_(g, g, value=1 - b2)
            p.addcdiv_(m, v.sqrt().add_(eps), value=-lr_t)


def fnv1a_trigram_ids(text_bytes: torch.Tensor, lengths: torch.Tensor, L: int, hash_size: int) -> torch.Tensor:
    """Reference for the device trigram hasher: ASCII bytes (N, Lmax) -> (N, L) ids, pad 0."""
    N = text_bytes.shape[0]
    out = torch.zeros(N, L, dtype=torch.int32)
    tb = text_bytes.to(torch.int64)
    for n in range(N):
        ln = int(lengths[n])
        for t in range(min(L, max(0, ln - 2))):
            h = 0x811C9DC5
            for j in range(3):
                h ^= int(tb[n, t + j])
                h = (h * 0x01000193) & _M32
            out[n, t] = 1 + h % (hash_size - 1)
    return out

"""Cosine-relevance softmax losses (K5-K7).

* ``dssm_explicit_loss``: reference parity head (1 positive + J explicit negatives per
  query; dssm_cnn_v2/cnn_dssm_th.py:159-182).  One fused HIP kernel computes loss, P and
  the gradients in a single pass.
* ``inbatch_loss``: every query against all M documents of the local batch.
  Flash-style HIP kernels: the (B x M) logits are never materialised (see
  csrc/kernels/loss.hip).
* ``cross_gpu_loss``: every query against the documents of ALL ranks.  The page
  vectors are all-gathered already in the kernels' bf16 padded layout (half the xGMI
  bytes of fp32), and the bf16 queries are gathered too (async, B*DP*2 bytes per rank).
  The backward then needs no reduce-scatter: dQ = local queries x all pages, and dD of
  the LOCAL pages = local pages x all W*B queries with the gathered per-query softmax
  scales (B floats per rank, gathered while the dQ kernel runs).  At W = 8 that replaces
  a reduce-scatter of an (M, DP) fp32 partial (~168 MB in, ~147 MB over xGMI per rank at
  B = 4096, J = 3) by ~2.6 MB of query gather; the FLOPs are the same.  The positive-pair
  term is applied to the local slice after.

Both take L2-normalised vectors (``ops.dense.l2_normalize``).
"""
from __future__ import annotations

import os
from typing import Optional, Tuple

import torch
import torch.distributed as dist

from . import reference as ref
from ._common import P, check, lib, stream, use_hip, use_hip_exact


class _ExplicitFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, qn, dn, gamma, clip):
        B, D = qn.shape
        J1 = dn.shape[1]
        q = qn.contiguous().float()
        d = dn.contiguous().float()
        loss = torch.empty(B, dtype=torch.float32, device=q.device)
        prob = torch.empty(B, dtype=torch.float32, device=q.device)
        dq = torch.empty_like(q)
        dd = torch.empty_like(d)
        check(lib().pv_dssm_explicit(P(q), P(d), P(loss), P(prob), P(dq), P(dd), B, J1, D, float(gamma), 1.0,
                                     int(clip), stream(q.device)), "pv_dssm_explicit")
        ctx.save_for_backward(dq, dd)
        ctx.mark_non_differentiable(prob)
        ctx.set_materialize_grads(False)  # no zero-filled gradients for prob / acc
        return loss, prob

    @staticmethod
    def backward(ctx, gl, _gp):
        if gl is None:
            return None, None, None, None
        dq, dd = ctx.saved_tensors
        g = gl.contiguous().float()
        return dq * g[:, None], dd * g[:, None, None], None, None


# limits of the fused explicit-loss kernel (pv_dssm_explicit: one wave per row, the query row
# and the 1+J raw cosines in registers; compile-time variants up to these)
EXPLICIT_MAX_J1 = 64
EXPLICIT_MAX_D = 1024


def dssm_explicit_loss(qn: torch.Tensor, dn: torch.Tensor, gamma: float, clip: bool = True
                       ) -> Tuple[torch.Tensor, torch.Tensor]:
    """qn (B, D), dn (B, 1+J, D) normalised -> (per-row loss (B,), P(D+|Q) (B,)).

    GPU: the fused HIP kernel (1+J <= 64, D <= 1024: covers the BERT tower's D = 768); beyond
    that the loss is rejected on the GPU rather than silently run as eager torch.  fp32 end to
    end, so it also runs at dtype="fp32" (``use_hip_exact``)."""
    if use_hip_exact(qn, dn):
        if dn.shape[1] > EXPLICIT_MAX_J1 or qn.shape[1] > EXPLICIT_MAX_D:
            raise NotImplementedError(f"explicit loss kernel supports 1+J <= {EXPLICIT_MAX_J1} and D <= "
                                      f"{EXPLICIT_MAX_D}; got 1+J = {dn.shape[1]}, D = {qn.shape[1]}")
        return _ExplicitFn.apply(qn, dn, float(gamma), bool(clip))
    R = torch.clamp((qn.unsqueeze(1) * dn).sum(-1), 0.0, 1.0) if clip else (qn.unsqueeze(1) * dn).sum(-1)
    e = torch.exp(gamma * R - gamma * R.max(dim=1, keepdim=True).values.detach())
    Pp = e[:, 0] / e.sum(dim=1)
    loss = -torch.log(torch.clamp(Pp, ref.BCE_EPS, 1.0 - ref.BCE_EPS))
    return loss, Pp.detach()


def _pad_bf16(x: torch.Tensor, DP: int) -> torch.Tensor:
    pre = getattr(x, "_pv_bf16", None)  # written by the L2-normalise kernel (ops/dense.py)
    if pre is not None and pre.shape == (x.shape[0], DP) and pre.device == x.device:
        return pre
    n, D = x.shape
    out = torch.zeros(n, DP, dtype=torch.bfloat16, device=x.device)
    out[:, :D] = x.detach()
    return out


def _ib_forward(qb: torch.Tensor, db: torch.Tensor, pos: torch.Tensor, B: int, M: int, DP: int, gamma: float,
                clip: int, with_dq: bool):
    """-> (per-row loss, P+, sumexp, U).  The positive logit first (ib_pos), then ONE pass
    over S whose row-sum kernel also finalises loss = g + log(sumexp) - spos and P+.
    When the query gradient will be needed, the same pass produces its normaliser-free
    part U (B, DP) (pv_ib_fwd_dq): the backward's dQ = scale * U."""
    s = stream(qb.device)
    L_ = lib()
    dev = qb.device
    spos = torch.empty(B, dtype=torch.float32, device=dev)
    check(L_.pv_ib_pos(P(qb), P(db), P(pos), P(spos), None, None, None, B, DP, float(gamma), int(clip), s), "pv_ib_pos")
    sumexp = torch.empty(B, dtype=torch.float32, device=dev)
    loss = torch.empty(B, dtype=torch.float32, device=dev)
    prob = torch.empty(B, dtype=torch.float32, device=dev)
    if not with_dq:
        part = torch.empty(L_.pv_ib_fwd_ws(B, M, DP), dtype=torch.float32, device=dev)
        check(L_.pv_ib_fwd(P(qb), P(db), P(sumexp), P(part), B, M, DP, float(gamma), int(clip), P(spos), P(loss),
                           P(prob), s), "pv_ib_fwd")
        return loss, prob, sumexp, None
    U = torch.empty(B, DP, dtype=torch.float32, device=dev)
    ws = torch.empty(max(L_.pv_ib_bwd_ws(B, M, DP), 1), dtype=torch.float32, device=dev)
    part = torch.empty(L_.pv_ib_fwd_dq_parts(B, M), dtype=torch.float32, device=dev)
    check(L_.pv_ib_fwd_dq(P(qb), P(db), P(sumexp), P(U), P(ws), P(part), B, M, DP, float(gamma), int(clip), P(spos),
                          P(loss), P(prob), s), "pv_ib_fwd_dq")
    return loss, prob, sumexp, U


def _loss_stats(loss: torch.Tensor, prob: torch.Tensor):
    """(mean loss, accuracy) as 0-dim device tensors from one kernel (loss.hip::loss_stats_kernel)."""
    lm = torch.empty((), dtype=torch.float32, device=loss.device)
    acc = torch.empty((), dtype=torch.float32, device=loss.device)
    check(lib().pv_loss_stats(P(loss), P(prob), loss.shape[0], P(lm), P(acc), stream(loss.device)), "pv_loss_stats")
    return lm, acc


def _grad_prologue(gl: torch.Tensor, reduce: bool, B: int, gamma: float, sumexp: torch.Tensor,
                   U: Optional[torch.Tensor], DP: int):
    """-> (softmax scale (B,), per-row upstream gradient (B,), dQ = scale * U or None) in one
    launch (loss.hip::ib_grad_scale_kernel); ``reduce``: gl is the mean loss's 0-dim gradient."""
    dev = sumexp.device
    g_in = gl.contiguous().float()
    scale = torch.empty(B, dtype=torch.float32, device=dev)
    grow = torch.empty(B, dtype=torch.float32, device=dev)
    dq = torch.empty(B, DP, dtype=torch.float32, device=dev) if U is not None else None
    check(lib().pv_ib_grad_scale(P(g_in), int(reduce), 1.0 / B, P(sumexp), B, float(gamma), P(U), DP, P(dq),
                                 P(scale), P(grow), stream(dev)), "pv_ib_grad_scale")
    return scale, grow, dq


FUSED_GLUE = True  # tests: False runs the round-5 glue launches (the fused path's oracle)


def _pos_inverse(pos: torch.Tensor, M: int, owner: Optional[torch.Tensor] = None) -> Optional[torch.Tensor]:
    """inv (M,) int32: the query whose positive page row m is, -1 for none; None when two queries
    share a positive (the fused dD finish needs a one-to-one map).  Cached on ``owner`` (the
    caller's index tensor, before any dtype conversion; the trainer keeps one per shape): a miss
    costs host syncs (min / max / unique); built eagerly, never inside a capture."""
    owner = pos if owner is None else owner
    key = (M, owner.data_ptr(), owner.numel(), owner.dtype)
    hit = getattr(owner, "_pv_inv", None)
    if hit is not None and hit[0] == key:
        return hit[1]
    if torch.cuda.is_current_stream_capturing():
        return None
    p = pos.long()
    inv = None
    if p.numel() == 0 or (int(p.min()) >= 0 and int(p.max()) < M and torch.unique(p).numel() == p.numel()):
        inv = torch.full((M,), -1, dtype=torch.int32, device=pos.device)
        inv[p] = torch.arange(p.numel(), dtype=torch.int32, device=pos.device)
    owner._pv_inv = (key, inv)
    return inv


class _InBatchFn(torch.autograd.Function):
    """Flash in-batch softmax loss.  Training (query gradient wanted): the fused ib7 forward + dQ
    part, ONE finish launch (positive logit, loss / P+, U, batch mean loss / accuracy), then in
    the backward the prologue with the query side of the positive pair folded in, the dD pass and
    ONE finish launch (split sum + the page side of the positive pair) — five glue launches of
    round 5 (ib_pos x 2, ib_rowsum, ib_split_reduce x 2 ... loss_stats) fold into the three."""

    @staticmethod
    def forward(ctx, qn, dn, pos, gamma, clip, reduce=False):
        B, D = qn.shape
        M = dn.shape[0]
        DP = (D + 31) // 32 * 32
        if DP > 192:
            raise ValueError("in-batch loss kernel supports D <= 192")
        qb = _pad_bf16(qn, DP)
        db = _pad_bf16(dn, DP)
        pos_in = pos
        pos = pos.to(torch.int32).contiguous()
        inv = _pos_inverse(pos, M, pos_in) if ctx.needs_input_grad[0] and FUSED_GLUE else None
        ctx.reduce = bool(reduce)
        ctx.meta = (B, M, D, DP, float(gamma), int(clip))
        if inv is not None:
            dev = qb.device
            L_ = lib()
            sumexp = torch.empty(B, dtype=torch.float32, device=dev)
            loss = torch.empty(B, dtype=torch.float32, device=dev)
            prob = torch.empty(B, dtype=torch.float32, device=dev)
            sraw = torch.empty(B, dtype=torch.float32, device=dev)
            U = torch.empty(B, DP, dtype=torch.float32, device=dev)
            ws = torch.empty(max(L_.pv_ib_bwd_ws(B, M, DP), 1), dtype=torch.float32, device=dev)
            part = torch.empty(L_.pv_ib_fwd_dq_parts(B, M), dtype=torch.float32, device=dev)
            lm = acc = bpart = None
            if reduce:
                lm = torch.empty((), dtype=torch.float32, device=dev)
                acc = torch.empty((), dtype=torch.float32, device=dev)
                bpart = torch.empty(2 * ((B + 3) // 4), dtype=torch.float32, device=dev)
            check(L_.pv_ib_fwd_dq2(P(qb), P(db), P(pos), P(sumexp), P(U), P(ws), P(part), B, M, DP, float(gamma),
                                   int(clip), P(sraw), P(loss), P(prob), P(bpart), P(lm), P(acc),
                                   stream(dev)), "pv_ib_fwd_dq2")
            ctx.save_for_backward(qb, db, pos, sumexp, U, sraw, inv)
            ctx.fused = True
        else:
            loss, prob, sumexp, U = _ib_forward(qb, db, pos, B, M, DP, gamma, clip, ctx.needs_input_grad[0])
            ctx.save_for_backward(qb, db, pos, sumexp, U)
            ctx.fused = False
            if reduce:
                lm, acc = _loss_stats(loss, prob)
        ctx.mark_non_differentiable(prob)
        ctx.set_materialize_grads(False)  # no zero-filled gradients for prob / acc
        if reduce:
            ctx.mark_non_differentiable(acc)
            return lm, prob, acc
        return loss, prob

    @staticmethod
    def backward(ctx, gl, _gp, _ga=None):
        if gl is None:  # materialize_grads is off: the loss output was not used
            return (None,) * len(ctx.needs_input_grad)
        B, M, D, DP, gamma, clip = ctx.meta
        if ctx.fused:
            qb, db, pos, sumexp, U, sraw, inv = ctx.saved_tensors
            dev = qb.device
            L_ = lib()
            s = stream(dev)
            g_in = gl.contiguous().float()
            scale = torch.empty(B, dtype=torch.float32, device=dev)
            grow = torch.empty(B, dtype=torch.float32, device=dev)
            dq = torch.empty(B, DP, dtype=torch.float32, device=dev)
            check(L_.pv_ib_grad_scale_pos(P(g_in), int(ctx.reduce), 1.0 / B, P(sumexp), B, gamma, P(U), DP, P(dq),
                                          P(scale), P(grow), P(db), P(pos), P(sraw), clip, s), "pv_ib_grad_scale_pos")
            dd = torch.empty(M, DP, dtype=torch.float32, device=dev)
            ws = torch.empty(max(L_.pv_ib_bwd_ws(M, B, DP), 1), dtype=torch.float32, device=dev)
            check(L_.pv_ib_bwd_dd_pos(P(db), P(qb), P(scale), P(dd), P(ws), M, B, DP, gamma, clip, P(inv), P(grow),
                                      P(sraw), s), "pv_ib_bwd_dd_pos")
            return dq[:, :D], dd[:, :D], None, None, None, None
        qb, db, pos, sumexp, U = ctx.saved_tensors
        s = stream(qb.device)
        L_ = lib()
        scale, g, dq = _grad_prologue(gl, ctx.reduce, B, gamma, sumexp, U, DP)
        dd = torch.empty(M, DP, dtype=torch.float32, device=qb.device)
        ws = torch.empty(max(L_.pv_ib_bwd_ws(M, B, DP), 1), dtype=torch.float32, device=qb.device)
        if U is None:
            dq = torch.empty(B, DP, dtype=torch.float32, device=qb.device)
            ws = torch.empty(max(L_.pv_ib_bwd_ws(B, M, DP), L_.pv_ib_bwd_ws(M, B, DP), 1),
                             dtype=torch.float32, device=qb.device)
            check(L_.pv_ib_bwd(P(qb), P(db), P(scale), P(dq), P(ws), B, M, DP, gamma, clip, 1, s), "pv_ib_bwd(dQ)")
        check(L_.pv_ib_bwd(P(db), P(qb), P(scale), P(dd), P(ws), M, B, DP, gamma, clip, 0, s), "pv_ib_bwd(dD)")
        check(L_.pv_ib_pos(P(qb), P(db), P(pos), None, P(g), P(dq), P(dd), B, DP, gamma, clip, s), "pv_ib_pos(bwd)")
        return dq[:, :D], dd[:, :D], None, None, None, None


# column-block size of the wide-vector path: B x ROWS_BLOCK_ELEMS / B fp32 logits per block
ROWS_BLOCK_ELEMS = 1 << 25


def _col_blocks(B: int, M: int):
    mb = max(256, min(M, ROWS_BLOCK_ELEMS // max(B, 1)))
    return [(c0, min(M, c0 + mb)) for c0 in range(0, M, mb)]


class _InBatchRowsFn(torch.autograd.Function):
    """Wide vectors (D > 192, e.g. BERT's 768; the narrow flash kernels hold D accumulators per
    query row in registers).  Default: the wide flash kernel (loss.hip::ibw_kernel, _wide_ok):
    S reduced over D across a workgroup's 4 waves, the gradient products on the same tile, no
    S block in HBM and no library GEMM.  Fallback (the widths ibw does not cover): the logits are
    tiled over page-column blocks at the GEMM level — each
    (B x Mb) block of S comes from a bf16 x bf16 -> fp32 library GEMM, is reduced by
    loss.hip::ib_rows_blk_kernel and dropped, so memory stays O(B * Mb) for any M; the
    backward recomputes each block (flash-style) and turns it into the block's dS in place.
    Positive pairs go through ib_pos as in the fused path."""

    @staticmethod
    def forward(ctx, qn, dn, pos, gamma, clip, reduce=False):
        B, D = qn.shape
        M = dn.shape[0]
        DP = (D + 31) // 32 * 32
        qb, db = _pad_bf16(qn, DP), _pad_bf16(dn, DP)
        pos = pos.to(torch.int32).contiguous()
        loss, prob, sumexp = _rows_forward(qb, db, pos, B, M, DP, gamma, clip)
        ctx.save_for_backward(qb, db, pos, sumexp)
        ctx.meta = (B, M, D, DP, float(gamma), int(clip))
        ctx.reduce = bool(reduce)
        ctx.mark_non_differentiable(prob)
        ctx.set_materialize_grads(False)
        if reduce:
            lm, acc = _loss_stats(loss, prob)
            ctx.mark_non_differentiable(acc)
            return lm, prob, acc
        return loss, prob

    @staticmethod
    def backward(ctx, gl, _gp, _ga=None):
        if gl is None:
            return (None,) * len(ctx.needs_input_grad)
        qb, db, pos, sumexp = ctx.saved_tensors
        B, M, D, DP, gamma, clip = ctx.meta
        dev, s, L_ = qb.device, stream(qb.device), lib()
        scale, g, _ = _grad_prologue(gl, ctx.reduce, B, gamma, sumexp, None, DP)
        dq = torch.zeros(B, DP, dtype=torch.float32, device=dev)
        dd = torch.empty(M, DP, dtype=torch.float32, device=dev)
        _rows_backward(qb, db, scale, gamma, clip, dq=dq, dd=dd)
        check(L_.pv_ib_pos(P(qb), P(db), P(pos), None, P(g), P(dq), P(dd), B, DP, gamma, clip, s), "pv_ib_pos(bwd)")
        return dq[:, :D], dd[:, :D], None, None, None, None


# Wide vectors on the flash kernel (loss.hip::ibw_kernel, DP % 128 == 0, 256..1024): no S block
# in HBM, no library GEMM; "0" = the column-block path below (fp32 S blocks + hipBLASLt)
IB_WIDE = True  # tests switch it off to exercise the column-block fallback at a covered width


def _wide_ok(DP: int) -> bool:
    return IB_WIDE and DP % 128 == 0 and 256 <= DP <= 1024 and DP not in (640, 896)


def _ibw(o, it, DP, scale, gamma, clip, mode, out):
    """loss.hip::pv_ibw: mode 0 row partial sums of o against it -> (splits, no) part; 1 / 2:
    out (no, DP) fp32 = the G-weighted sums of it rows (scale by o row / by it row)."""
    no, ni = o.shape[0], it.shape[0]
    L_ = lib()
    ws_n = L_.pv_ibw_ws(no, ni, DP) if mode else 0
    ws = torch.empty(max(ws_n, 1), dtype=torch.float32, device=o.device) if ws_n else None
    check(L_.pv_ibw(P(o), no, P(it), ni, DP, P(scale), float(gamma), int(clip), mode, P(out), P(ws),
                    stream(o.device)), f"pv_ibw(mode {mode})")
    return out


def _rows_forward(qb, db, pos, B, M, DP, gamma, clip):
    """Wide-vector forward over page-column blocks -> (per-row loss, P+, sumexp)."""
    dev, s, L_ = qb.device, stream(qb.device), lib()
    spos = torch.empty(B, dtype=torch.float32, device=dev)
    check(L_.pv_ib_pos(P(qb), P(db), P(pos), P(spos), None, None, None, B, DP, float(gamma), int(clip), s),
          "pv_ib_pos")
    if _wide_ok(DP):
        ns = int(L_.pv_ibw_splits(B, M))
        part = _ibw(qb, db, DP, None, gamma, clip, 0, torch.empty(ns, B, dtype=torch.float32, device=dev))
        sumexp = torch.empty(B, dtype=torch.float32, device=dev)
        loss = torch.empty(B, dtype=torch.float32, device=dev)
        prob = torch.empty(B, dtype=torch.float32, device=dev)
        check(L_.pv_ib_rowsum(P(part), P(sumexp), B, ns, P(spos), P(loss), P(prob), float(gamma), s), "pv_ib_rowsum")
        return loss, prob, sumexp
    blocks = _col_blocks(B, M)
    part = torch.empty(len(blocks), B, dtype=torch.float32, device=dev)
    for k, (c0, c1) in enumerate(blocks):
        S = torch.mm(qb, db[c0:c1].t(), out_dtype=torch.float32)
        check(L_.pv_ib_rows_blk(P(S), c1 - c0, B, c1 - c0, None, P(part[k]), float(gamma), int(clip), s),
              "pv_ib_rows_blk")
    sumexp = torch.empty(B, dtype=torch.float32, device=dev)
    loss = torch.empty(B, dtype=torch.float32, device=dev)
    prob = torch.empty(B, dtype=torch.float32, device=dev)
    check(L_.pv_ib_rowsum(P(part), P(sumexp), B, len(blocks), P(spos), P(loss), P(prob), float(gamma), s),
          "pv_ib_rowsum")
    return loss, prob, sumexp


def _rows_backward(xb, yb, scale, gamma, clip, dq=None, dd=None):
    """Flash-style wide-vector backward of the (R x C) logits of rows xb against columns yb,
    recomputed per column block: dS = rows_blk(S, per-row scale); dq += dS yb (rows' gradient,
    accumulated), dd[block] = dS^T xb (columns' gradient, written)."""
    R, C = xb.shape[0], yb.shape[0]
    s, L_ = stream(xb.device), lib()
    DP = xb.shape[1]
    if _wide_ok(DP):  # flash passes: dq rows own, walk the columns; dd columns own, walk the rows
        if dq is not None:  # written, not accumulated: every caller passes a zeroed dq
            _ibw(xb, yb, DP, scale, gamma, clip, 1, dq)
        if dd is not None:
            _ibw(yb, xb, DP, scale, gamma, clip, 2, dd)
        return
    for c0, c1 in _col_blocks(R, C):
        S = torch.mm(xb, yb[c0:c1].t(), out_dtype=torch.float32)
        check(L_.pv_ib_rows_blk(P(S), c1 - c0, R, c1 - c0, P(scale), None, float(gamma), int(clip), s),
              "pv_ib_rows_blk(dS)")
        dS = S.to(torch.bfloat16)
        if dq is not None:
            dq += torch.mm(dS, yb[c0:c1], out_dtype=torch.float32)
        if dd is not None:
            dd[c0:c1] = torch.mm(dS.t(), xb, out_dtype=torch.float32)


class PageGather:
    """An in-flight all-gather of the local page vectors in the loss kernels' bf16 padded
    layout, started as soon as the doc tower is done so that RCCL overlaps the query
    tower's forward; consumed by cross_gpu_loss."""

    def __init__(self, dn: torch.Tensor, group=None):
        W = dist.get_world_size(group)
        self.D = dn.shape[1]
        self.DP = (self.D + 31) // 32 * 32
        self.dbl = _pad_bf16(dn, self.DP)
        self.db = torch.empty(dn.shape[0] * W, self.DP, dtype=torch.bfloat16, device=dn.device)
        self.work = dist.all_gather_into_tensor(self.db, self.dbl, group=group, async_op=True)
        self.source = dn

    def wait(self):
        if self.work is not None:
            self.work.wait()
            self.work = None
        return self.dbl, self.db


def start_page_gather(dn: torch.Tensor, group=None) -> Optional[PageGather]:
    """Begin the cross-GPU page-vector gather early (None when it does not apply)."""
    from ..parallel.dist import active
    if not active(group) or not use_hip(dn):
        return None
    return PageGather(dn, group)


class _CrossGpuFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, qn, dn, pos_local, gamma, clip, group, pre, reduce=False):
        W = dist.get_world_size(group)
        rank = dist.get_rank(group)
        B, D = qn.shape
        n = dn.shape[0]
        M = n * W
        DP = (D + 31) // 32 * 32
        qb = _pad_bf16(qn, DP)
        if pre is not None:
            dbl, db = pre.wait()
        else:
            dbl = _pad_bf16(dn, DP)
            db = torch.empty(M, DP, dtype=torch.bfloat16, device=qn.device)
            dist.all_gather_into_tensor(db, dbl, group=group)
        pos_local = pos_local.to(torch.int32).contiguous()
        pos = (pos_local + rank * n).contiguous()
        loss, prob, sumexp, U = _ib_forward(qb, db, pos, B, M, DP, gamma, clip, ctx.needs_input_grad[0])
        ctx.mark_non_differentiable(prob)
        ctx.set_materialize_grads(False)  # no zero-filled gradients for prob / acc
        # the backward scores the LOCAL pages against ALL ranks' queries (dD needs no
        # cross-rank sum then): gather the bf16 queries now, in flight during the rest of
        # the forward and the tower's own backward (B*DP*2 bytes per rank)
        qall = torch.empty(B * W, DP, dtype=torch.bfloat16, device=qn.device)
        ctx.qwork = dist.all_gather_into_tensor(qall, qb, group=group, async_op=True)
        # a plain attribute, not a saved tensor: the in-flight collective writes qall after
        # this point (gloo copies the result back on completion, bumping its version)
        ctx.qall = qall
        ctx.save_for_backward(qb, db, dbl, pos_local, sumexp, U)
        ctx.meta = (B, M, n, D, DP, float(gamma), int(clip), group, W)
        ctx.reduce = bool(reduce)
        if reduce:
            lm, acc = _loss_stats(loss, prob)
            ctx.mark_non_differentiable(acc)
            return lm, prob, acc
        return loss, prob

    @staticmethod
    def backward(ctx, gl, _gp, _ga=None):
        if gl is None:  # materialize_grads is off: the loss output was not used
            return (None,) * len(ctx.needs_input_grad)
        qb, db, dbl, pos_local, sumexp, U = ctx.saved_tensors
        B, M, n, D, DP, gamma, clip, group, W = ctx.meta
        s = stream(qb.device)
        L_ = lib()
        scale, g, dq = _grad_prologue(gl, ctx.reduce, B, gamma, sumexp, U, DP)
        # every rank's per-query softmax scale (B floats each), gathered while dQ runs
        scale_all = torch.empty(B * W, dtype=torch.float32, device=qb.device)
        swork = dist.all_gather_into_tensor(scale_all, scale, group=group, async_op=True)
        dd = torch.empty(n, DP, dtype=torch.float32, device=qb.device)
        ws = torch.empty(max(L_.pv_ib_bwd_ws(B, M, DP), L_.pv_ib_bwd_ws(n, B * W, DP), 1),
                         dtype=torch.float32, device=qb.device)
        if U is None:  # (else the forward already summed exp * clip' * d over ALL ranks' pages)
            dq = torch.empty(B, DP, dtype=torch.float32, device=qb.device)
            check(L_.pv_ib_bwd(P(qb), P(db), P(scale), P(dq), P(ws), B, M, DP, gamma, clip, 1, s), "pv_ib_bwd(dQ)")
        ctx.qwork.wait()
        ctx.qwork = None
        qall, ctx.qall = ctx.qall, None
        swork.wait()
        # dD of the local pages = sum over all W*B queries: no reduce-scatter of an (M, DP)
        # fp32 partial (W x the bytes of dd) over xGMI
        check(L_.pv_ib_bwd(P(dbl), P(qall), P(scale_all), P(dd), P(ws), n, B * W, DP, gamma, clip, 0, s),
              "pv_ib_bwd(dD)")
        check(L_.pv_ib_pos(P(qb), P(dbl), P(pos_local), None, P(g), P(dq), P(dd), B, DP, gamma, clip, s),
              "pv_ib_pos(bwd)")
        return dq[:, :D], dd[:, :D], None, None, None, None, None, None


class _CrossGpuRowsFn(torch.autograd.Function):
    """Cross-GPU negatives for wide vectors (D > 192: BERT's 768) with the same communication
    design as _CrossGpuFn — the page gather started after the doc tower, the bf16 queries and
    the per-query softmax scales gathered asynchronously, and NO reduce-scatter in backward:
    dQ = local queries x all pages, dD of the LOCAL pages = all W*B queries x local pages.  The
    passes (_rows_forward / _rows_backward) run on the ``ibw`` flash kernel (loss.hip, DP a
    multiple of 128 in 256..1024: the row's d-slices split over a workgroup's 4 waves, no logits
    in HBM); only the widths ibw does not cover fall back to column blocks of library-GEMM
    logits."""

    @staticmethod
    def forward(ctx, qn, dn, pos_local, gamma, clip, group, pre, reduce=False):
        W = dist.get_world_size(group)
        rank = dist.get_rank(group)
        B, D = qn.shape
        n = dn.shape[0]
        M = n * W
        DP = (D + 31) // 32 * 32
        qb = _pad_bf16(qn, DP)
        if pre is not None:
            dbl, db = pre.wait()
        else:
            dbl = _pad_bf16(dn, DP)
            db = torch.empty(M, DP, dtype=torch.bfloat16, device=qn.device)
            dist.all_gather_into_tensor(db, dbl, group=group)
        pos_local = pos_local.to(torch.int32).contiguous()
        pos = (pos_local + rank * n).contiguous()
        loss, prob, sumexp = _rows_forward(qb, db, pos, B, M, DP, gamma, clip)
        ctx.mark_non_differentiable(prob)
        ctx.set_materialize_grads(False)
        qall = torch.empty(B * W, DP, dtype=torch.bfloat16, device=qn.device)
        ctx.qwork = dist.all_gather_into_tensor(qall, qb, group=group, async_op=True)
        ctx.qall = qall
        ctx.save_for_backward(qb, db, dbl, pos_local, sumexp)
        ctx.meta = (B, M, n, D, DP, float(gamma), int(clip), group, W)
        ctx.reduce = bool(reduce)
        if reduce:
            lm, acc = _loss_stats(loss, prob)
            ctx.mark_non_differentiable(acc)
            return lm, prob, acc
        return loss, prob

    @staticmethod
    def backward(ctx, gl, _gp, _ga=None):
        if gl is None:
            return (None,) * len(ctx.needs_input_grad)
        qb, db, dbl, pos_local, sumexp = ctx.saved_tensors
        B, M, n, D, DP, gamma, clip, group, W = ctx.meta
        dev, s, L_ = qb.device, stream(qb.device), lib()
        scale, g, _ = _grad_prologue(gl, ctx.reduce, B, gamma, sumexp, None, DP)
        scale_all = torch.empty(B * W, dtype=torch.float32, device=dev)
        swork = dist.all_gather_into_tensor(scale_all, scale, group=group, async_op=True)
        dq = torch.zeros(B, DP, dtype=torch.float32, device=dev)
        _rows_backward(qb, db, scale, gamma, clip, dq=dq)  # local queries x all pages
        ctx.qwork.wait()
        ctx.qwork = None
        qall, ctx.qall = ctx.qall, None
        swork.wait()
        dd = torch.empty(n, DP, dtype=torch.float32, device=dev)
        _rows_backward(qall, dbl, scale_all, gamma, clip, dd=dd)  # all queries x local pages
        check(L_.pv_ib_pos(P(qb), P(dbl), P(pos_local), None, P(g), P(dq), P(dd), B, DP, gamma, clip, s),
              "pv_ib_pos(bwd)")
        return dq[:, :D], dd[:, :D], None, None, None, None, None, None


def _reduce_rows(loss: torch.Tensor, prob: torch.Tensor):
    return loss.mean(), prob, (prob > 0.5).float().mean()


# The in-batch kernels shift every logit by the largest possible one (gamma; no running max):
# exp(gamma * (S - 1)) must stay a normal fp32 for the lowest S (0 with the clip, -1 without),
# i.e. gamma * span <= ~87.  Larger scales would underflow whole rows to 0 (log 0 = -inf).
MAX_LOGIT_SPAN = 80.0


def _check_gamma(gamma: float, clip: bool) -> None:
    span = float(gamma) * (1.0 if clip else 2.0)
    if span > MAX_LOGIT_SPAN:
        raise ValueError(f"in-batch softmax scale {gamma} too large (gamma * logit span {span:.0f} > "
                         f"{MAX_LOGIT_SPAN:.0f}: exp underflows in fp32)")


def cross_gpu_loss(qn: torch.Tensor, dn: torch.Tensor, pos_local: torch.Tensor, gamma: float, clip: bool = True,
                   group=None, gathered: Optional[PageGather] = None, reduce: bool = False):
    """qn (B, D) and the LOCAL page vectors dn (n, D), normalised; pos_local (B,) indexes dn.
    Every query is scored against the pages of all ranks (rank r's pages at rows r*n...).
    ``gathered``: the PageGather started on ``dn`` right after the doc tower.
    -> (per-row loss, P+); ``reduce``: (mean loss, P+, accuracy), the mean and metric
    computed in the loss kernels' epilogue (no separate reductions)."""
    _check_gamma(gamma, clip)
    from ..parallel.dist import active
    if not active(group):
        return inbatch_loss(qn, dn, pos_local, gamma, clip, reduce=reduce)
    if use_hip(qn, dn):
        if gathered is not None and gathered.source is not dn:
            raise ValueError("the prefetched gather belongs to another page tensor")
        fn = _CrossGpuFn if qn.shape[1] <= 192 else _CrossGpuRowsFn
        return fn.apply(qn, dn, pos_local, float(gamma), bool(clip), group, gathered, bool(reduce))
    from ..parallel.dist import all_gather_autograd
    docs = all_gather_autograd(dn)
    pos = pos_local + dist.get_rank(group) * dn.shape[0]
    return inbatch_loss(qn, docs, pos, gamma, clip, reduce=reduce)


def inbatch_loss(qn: torch.Tensor, dn: torch.Tensor, pos_index: torch.Tensor, gamma: float, clip: bool = True,
                 reduce: bool = False):
    """qn (B, D), dn (M, D) normalised; pos_index (B,) -> (per-row loss, P_pos);
    ``reduce``: (mean loss, P_pos, accuracy)."""
    _check_gamma(gamma, clip)
    if use_hip(qn, dn):
        if qn.shape[1] > 192:
            return _InBatchRowsFn.apply(qn, dn, pos_index, float(gamma), bool(clip), bool(reduce))
        return _InBatchFn.apply(qn, dn, pos_index, float(gamma), bool(clip), bool(reduce))
    out = ref.inbatch_softmax_loss(qn, dn, pos_index, gamma, clip)
    return _reduce_rows(*out) if reduce else out

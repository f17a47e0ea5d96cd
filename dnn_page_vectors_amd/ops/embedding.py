"""Embedding bag (sum / mean of token rows) for the DSSM MLP tower, and the device
trigram hasher (K0).

Two execution plans for ``bag = scale * onehot_counts(ids) @ W``:

* ``gather``  — HIP kernel gathers W rows per token (bf16 rows, one wave per bag); best for
  short bags (queries) and inference;
* ``counts``  — HIP kernel builds the dense count matrix C (N x V, bf16), then one
  hipBLASLt GEMM C @ W on the matrix cores; the backward is the GEMM C^T @ dY (no
  scatter atomics at all).  For 2k-token pages at V = 30k, E = 512 this is ~0.13 TFLOP
  of MFMA instead of ~8 GB of row gathers (fwd) + ~16 GB of float atomics (bwd).

Backward: the counts GEMM C^T @ dY for the counts plan; for the gather plan (short bags,
V < 65535) a sparse path — the forward also emits 16-bit sort keys (token id, pad -> V),
the backward sorts the N*L (token, slot) entries and ``pv_bag_bwd_sorted`` sums each
token's run of dY rows into dW (MLP query tower, N 4096 x L 45: ~0.19 ms of counts build +
126 GFLOP GEMM replaced by a 184k-entry sort + ~0.4 GB of row reads).  CPU: plain torch.
"""
from __future__ import annotations

import contextlib
import os
from typing import Optional

import torch

from . import dense as dops
from . import grad_sink
from . import reference as ref
from ._common import P, check, lib, stream, use_hip
from ..parallel.sparse_rows import note_rows
from .conv_pool import sort_pairs_iota


_HIST_MAX = 38912  # csrc/kernels/embedding.hip HIST_MAX


def _counts(ids: torch.Tensor, V: int, pad: int):
    N, L = ids.shape
    ldc = (V + 63) // 64 * 64
    # the LDS-histogram kernels write every element (ldc % 64 == 0; vocabularies wider than
    # _HIST_MAX in windows of it): no zero fill
    C = torch.empty(N, ldc, dtype=torch.bfloat16, device=ids.device)
    lens = torch.empty(N, dtype=torch.float32, device=ids.device)
    check(lib().pv_bag_counts(P(ids), P(C), P(lens), N, L, V, ldc, pad, 0, stream(ids.device)),
          "pv_bag_counts")
    return C, lens


def _counts8(ids: torch.Tensor, V: int, pad: int, want16: bool):
    """-> (e4m3 counts (N, ldc8), bf16 counts (N, ldc16) or None, lens): one histogram kernel
    (embedding.hip::bag_counts8_kernel); ldc8 is the MX GEMM's K padding (multiple of 128)."""
    from .fp8 import MX_BK

    N, L = ids.shape
    ldc8 = -(-V // MX_BK) * MX_BK
    ldc16 = (V + 63) // 64 * 64
    C8 = torch.empty(N, ldc8, dtype=torch.uint8, device=ids.device)
    C16 = torch.empty(N, ldc16, dtype=torch.bfloat16, device=ids.device) if want16 else None
    lens = torch.empty(N, dtype=torch.float32, device=ids.device)
    check(lib().pv_bag_counts8(P(ids), P(C16), ldc16, P(C8), ldc8, P(lens), N, L, V, pad, stream(ids.device)),
          "pv_bag_counts8")
    return C8, C16, lens


def _counts_gemm(C: torch.Tensor, W16: torch.Tensor, lens: Optional[torch.Tensor] = None,
                 bias: Optional[torch.Tensor] = None, act: str = "none") -> torch.Tensor:
    """C (N, V) @ W16 (V, E) in fp32.  The (N, E) output has only (N/256)(E/256) = 32 tiles for
    the MLP page bags (N 4096, E 512) over a 30000-long reduction, so the single GEMM runs on
    a fraction of the CUs; split V into 8 batched fp32-output GEMMs and sum the partials:
    0.293 -> 0.148 ms (tools/bag_gemm_micro.py), and the result is no longer rounded to bf16."""
    N, V = C.shape
    E = W16.shape[1]
    sk = _BAG_SPLITK or next((k for k in (8, 4, 2) if V % k == 0 and V // k >= 2048), 1)
    if V % sk:
        sk = 1
    if sk > 1 and N * E <= 8 * 1024 * 1024:
        try:
            Cb = C.unflatten(1, (sk, V // sk)).transpose(0, 1)
            part = torch.bmm(Cb, W16.reshape(sk, V // sk, E), out_dtype=torch.float32)
        except (TypeError, RuntimeError, NotImplementedError):
            part = None
        if part is not None:  # split-K sum fused with the bag-mean 1/len / bias / activation
            return dops.colsum(part, scale=lens, bias=bias, act=act, scale_is_len=True)
    out = (C @ W16).float()
    if lens is not None:
        out = out / lens.clamp(min=1.0)[:, None]
    if bias is not None:
        out = out + bias.float()
    return dops._torch_act(out, act)


# Long bags (the counts plan): the dense N x V bf16 count matrix (one LDS-histogram kernel)
# times W.  "lib" = hipBLASLt GEMMs; "dense" (round 6) = in-tree MFMA kernels that stream both
# operands by LDS-DMA (bag_gemm.hip bagd_mm_kernel): forward C W and weight gradient (Gt C)^T.
# Measured (profiles/r6/bagd/): the eager MLP step 1.485 -> 1.356 and 1.294 -> 1.207 ms (same
# process, two boxes: the library calls' host cost sits on the step), but inside a captured graph
# the library kernels are faster (160 + 129 vs 172 + 152 us; bench 1.033-1.050 vs 1.063-1.072
# ms alternated on one box).  "auto" (default): dense for eager steps, lib inside a graph.  (The
# round-5 segment-list arm — count tiles built in LDS from per-atom lists — lost to both on the
# list build, 300 vs 45-58 us, and its weight gradient, 243 us, and was removed in round 6:
# profiles/r5_bag/.)
BAG_GEMM = os.environ.get("PAGEVEC_BAG_GEMM", "auto")


_BAG_SCOPE = [None]


@contextlib.contextmanager
def bag_gemm_scope(plan: Optional[str]):
    """Fix the "auto" choice for a block (the trainer: "lib" for graph-mode trainers, whose eager
    warm-up steps must initialise the library before the capture)."""
    prev, _BAG_SCOPE[0] = _BAG_SCOPE[0], plan
    try:
        yield
    finally:
        _BAG_SCOPE[0] = prev


def _bag_gemm() -> str:
    if BAG_GEMM != "auto":
        return BAG_GEMM
    if _BAG_SCOPE[0] is not None:
        return _BAG_SCOPE[0]
    return "lib" if torch.cuda.is_current_stream_capturing() else "dense"


def _dense_ok(C: torch.Tensor, W16: torch.Tensor, V: int, E: int) -> bool:
    return (_bag_gemm() == "dense" and E % 8 == 0 and C.dtype == torch.bfloat16 and C.shape[1] % 64 == 0
            and W16 is not None and W16.dtype == torch.bfloat16 and W16.is_contiguous() and tuple(W16.shape) == (V, E))


def _dense_forward_partials(C: torch.Tensor, W16: torch.Tensor, V: int) -> torch.Tensor:
    """(splits, N, E) fp32 partial products C[:, slice] @ W16[slice] on bagd_mm_kernel (~256
    workgroups: split-K over the vocabulary)."""
    N, ldc = C.shape
    E = W16.shape[1]
    tiles = -(-N // 256) * -(-E // 128)
    want = max(1, min(ldc // 64, round(256 / tiles)))
    ns = int(lib().pv_bagd_splits(N, V, E, ldc, want))
    part = torch.empty(ns, N, E, dtype=torch.float32, device=C.device)
    check(lib().pv_bagd_fwd(P(C), ldc, P(W16), P(part), N, V, E, want, stream(C.device)), "pv_bagd_fwd")
    return part


def _dense_weight_grad(C: torch.Tensor, gs: torch.Tensor, V: int, out: torch.Tensor) -> None:
    """out (V, E) fp32 (row stride out.stride(0)) = C[:, :V]^T gs on bagd_mm_kernel (gs (N, E) bf16
    transposed to a zero-padded (E, ceil64(N)) scratch first)."""
    N, ldc = C.shape
    E = gs.shape[1]
    Np = -(-N // 64) * 64
    ws = torch.empty(E, Np, dtype=torch.bfloat16, device=C.device)
    check(lib().pv_bagd_wgrad(P(C), ldc, P(gs.contiguous()), P(ws), P(out), int(out.stride(0)), 0, N, V, E,
                              stream(C.device)), "pv_bagd_wgrad")


SPARSE_BWD = os.environ.get("PAGEVEC_BAG_SPARSE_BWD", "1") != "0"
_BAG_SPLITK = int(os.environ.get("PAGEVEC_BAG_SPLITK", "0"))  # override of the vocabulary split (A/B)
BAG_EPW = int(os.environ.get("PAGEVEC_BAG_EPW", "64"))  # sorted entries per wave (>= 8)
FP8_BAG = os.environ.get("PAGEVEC_FP8_BAG", "1") != "0"  # 0: fp8 towers keep the bf16 counts GEMM (A/B)
# fp8 bag weight gradient: C^T G on the MX fp8 MFMA too (e4m3 counts transposed, G per-tensor
# scaled e4m3) instead of the exact bf16 counts + hipBLASLt.  Opt-in: the product is within
# ~8 % of the exact gradient (per-row gradients below amax * 2^-9 / 448 flush to zero), and
# the step-level A/B did not show a gain (chunked 1.737 vs 1.683 ms median,
# profiles/r5_lt/chunked_fp8bwd_ab.txt) although the isolated micro is faster
FP8_BWD = os.environ.get("PAGEVEC_FP8_BWD", "0") != "0"


_BAG_ACT = {"none": 0, "relu": 1, "tanh": 3}


class _BagFn(torch.autograd.Function):
    """act(scale * counts(ids) @ W + bias): the bag, its mean, and (optionally) the MLP
    tower's first bias + activation in the producing kernel (gather epilogue / split-K sum
    epilogue); the backward runs the activation mask, the bias column sum and dW."""

    @staticmethod
    def forward(ctx, ids, W, W16, pad, mean, plan, bias, act, w8=None):
        ids = ids.to(torch.int32).contiguous()
        N, L = ids.shape
        V, E = W.shape
        ctx.V = V
        ctx.W = W  # the parameters themselves (flat-gradient direct-write targets)
        ctx.bias = bias
        ctx.act = act
        ctx.mean = bool(mean)
        bf = bias.float().contiguous() if bias is not None else None
        C = None
        if plan == "gather":
            # short bags: row gather forward; the backward is sparse (sort the (token, slot)
            # entries, sum each token's run of dY rows) -- no N x V counts matrix at all
            sparse = SPARSE_BWD and V < 65535 and E % 4 == 0 and N * L < (1 << 31)
            want_keys = sparse and ctx.needs_input_grad[1]
            out = torch.empty(N, E, dtype=torch.float32, device=ids.device)
            lens = torch.empty(N, dtype=torch.float32, device=ids.device)
            keys = torch.empty(N * L, dtype=torch.int16, device=ids.device) if want_keys else None
            check(lib().pv_embedding_bag(P(ids), P(W16), P(out), P(lens), P(keys), P(bf), _BAG_ACT[act], N, L, E, V,
                                         pad, int(mean), stream(ids.device)), "pv_embedding_bag")
            if not want_keys and ctx.needs_input_grad[1]:
                C, lens = _counts(ids, V, pad)
        elif w8 is not None:
            # fp8 bag (use_fp8 towers): e4m3 counts x the step's e4m3 W^T on the block-scaled
            # MFMA, split-K partials reduced with the mean / bias / activation epilogue; the
            # exact bf16 counts are kept only for the weight gradient (C^T G, bf16)
            from . import fp8 as fops

            W8t, amax = w8
            want = ctx.needs_input_grad[1]
            fp8_bwd = want and FP8_BWD and E % 4 == 0
            C8, C, lens = _counts8(ids, V, pad, want and not fp8_bwd)
            if C is not None and not fp8_bwd and _bag_gemm() == "dense" and E % 8 == 0 and C.shape[1] % 64 == 0:
                ctx.dense = True  # the bf16 weight gradient C^T G on bagd_mm_kernel
            if fp8_bwd:  # the e4m3 counts serve the weight gradient too (no bf16 N x V matrix)
                C = C8
                ctx.fp8_bwd = True
            part = fops.gemm_mx8(C8, W8t, 1.0 / fops.FP8_MAX, amax)
            if part.dim() == 2:
                part = part.unsqueeze(0)
            out = dops.colsum(part, scale=lens if mean else None, bias=bf, act=act, scale_is_len=True)
            keys = None
        else:
            C, lens = _counts(ids, V, pad)
            if _dense_ok(C, W16, V, E):  # in-tree MFMA product, split-K partials + fused epilogue
                out = dops.colsum(_dense_forward_partials(C, W16, V), scale=lens if mean else None, bias=bf,
                                  act=act, scale_is_len=True)
                ctx.dense = True
            else:
                out = _counts_gemm(C[:, :V], W16, lens if mean else None, bf, act)
            keys = None
        ctx.sparse = (L, E) if C is None else None
        ctx.save_for_backward(keys if C is None else C, lens, out if act != "none" else None)
        return out

    @staticmethod
    def backward(ctx, g):
        W, V, bias = ctx.W, ctx.V, ctx.bias
        first, lens, y = ctx.saved_tensors
        g = g.contiguous().float()
        if ctx.sparse is None and ctx.needs_input_grad[1]:
            return _counts_backward(ctx, g, first, lens, y)
        if y is not None:  # activation mask: dpre = dy * act'(y)
            dz = torch.empty_like(g)
            check(lib().pv_act_bwd(P(y), P(g), P(dz), g.numel(), _BAG_ACT[ctx.act], stream(g.device)), "pv_act_bwd")
            g = dz
        db = None
        if bias is not None and ctx.needs_input_grad[6]:
            tb = grad_sink.write_target(bias)
            db = dops.colsum(g, out=tb, accumulate=tb is not None)  # a first contribution's region is zero
            if tb is not None:
                grad_sink.done(bias)
                db = None
            elif db.dtype != bias.dtype:
                db = db.to(bias.dtype)
        if not ctx.needs_input_grad[1]:
            return None, None, None, None, None, None, db, None, None
        if ctx.sparse is not None:
            keys = first
            L, E = ctx.sparse
            M = keys.numel()
            skeys = torch.empty_like(keys)
            svals = torch.empty(M, dtype=torch.int32, device=keys.device)
            sort_pairs_iota(keys, skeys, svals, max(1, int(V).bit_length()))
            tw = grad_sink.accum_target(W)  # the kernel accumulates atomically
            dW = tw if tw is not None else torch.zeros(V, E, dtype=torch.float32, device=keys.device)
            check(lib().pv_bag_bwd_sorted(P(skeys), P(svals), P(g), P(lens), P(dW), M, BAG_EPW, L, E, V,
                                          int(ctx.mean), stream(g.device)), "pv_bag_bwd_sorted")
            if tw is not None:
                grad_sink.done(W)
                dW = None
            return None, dW, None, None, None, None, db, None, None
        C = first
        scale = (1.0 / lens.clamp(min=1.0)) if ctx.mean else torch.ones_like(lens)
        gs = (g * scale[:, None]).to(torch.bfloat16)
        Ct = C[:, :V].t()
        tw = grad_sink.write_target(W)  # fp32-output GEMM straight into the flat gradient
        if tw is not None:
            try:
                torch.mm(Ct, gs, out_dtype=torch.float32, out=tw)
            except (TypeError, RuntimeError, NotImplementedError):
                tw.copy_(Ct @ gs)
            grad_sink.done(W)
            return None, None, None, None, None, None, db, None, None
        return None, (Ct @ gs).float(), None, None, None, None, db, None, None


def _counts_backward(ctx, g, C, lens, y):
    """Backward of the counts-GEMM bag (long bags): ONE prologue kernel computes the
    activation mask, the fp32 dz for the bias column sum and bf16(dz / len) for the C^T G
    weight-gradient GEMM (was act_bwd + clamp + reciprocal + mul + cast)."""
    W, V, bias = ctx.W, ctx.V, ctx.bias
    N, E = g.shape
    want_db = bias is not None and ctx.needs_input_grad[6]
    fp8_bwd = getattr(ctx, "fp8_bwd", False)
    dz = torch.empty_like(g) if want_db or fp8_bwd else None
    gs = torch.empty(N, E, dtype=torch.bfloat16, device=g.device)
    check(lib().pv_act_bwd_rowscale(P(y), P(g), P(dz), P(gs), P(lens) if ctx.mean else None, E, g.numel(),
                                    _BAG_ACT[ctx.act] if y is not None else 0, stream(g.device)),
          "pv_act_bwd_rowscale")
    db = None
    if want_db:
        tb = grad_sink.write_target(bias)
        db = dops.colsum(dz, out=tb, accumulate=tb is not None)
        if tb is not None:
            grad_sink.done(bias)
            db = None
        elif db.dtype != bias.dtype:
            db = db.to(bias.dtype)
    if fp8_bwd:  # e4m3 C^T x e4m3 G on the MX fp8 MFMA
        tw = grad_sink.write_target(W)
        dW = tw if tw is not None else torch.empty(V, E, dtype=torch.float32, device=g.device)
        _fp8_weight_grad(C, dz, V, dW, lens if ctx.mean else None)
        if tw is not None:
            grad_sink.done(W)
            dW = None
        return None, dW, None, None, None, None, db, None, None
    if getattr(ctx, "dense", False):  # bag_gemm.hip bagd_mm_kernel: (Gt C)^T stored as dW rows
        tw = grad_sink.write_target(W)
        if tw is not None and tw.is_contiguous() and tw.data_ptr() % 16 == 0:
            _dense_weight_grad(C, gs, V, tw)
            grad_sink.done(W)
            return None, None, None, None, None, None, db, None, None
        if tw is None:
            dW = torch.empty(V, gs.shape[1], dtype=torch.float32, device=g.device)
            _dense_weight_grad(C, gs, V, dW)
            return None, dW, None, None, None, None, db, None, None
    Ct = C[:, :V].t()
    tw = grad_sink.write_target(W)  # fp32-output GEMM straight into the flat gradient
    if tw is not None:
        try:
            torch.mm(Ct, gs, out_dtype=torch.float32, out=tw)
        except (TypeError, RuntimeError, NotImplementedError):
            tw.copy_(Ct @ gs)
        grad_sink.done(W)
        return None, None, None, None, None, None, db, None, None
    return None, (Ct @ gs).float(), None, None, None, None, db, None, None


def _fp8_weight_grad(C8, dz, V, out, lens=None):
    """out (V, E) fp32 = C8[:, :V]^T (dz / len) on the MX fp8 MFMA: the counts (exact e4m3 up to
    16, the forward's own operand) transposed to K(page)-contiguous rows, the row-scaled fp32
    gradient quantised per tensor to e4m3 and transposed, one gemm_mx8 with the dequant scale
    amax_g / 448 in its epilogue.  Reference: the exact bf16 C^T G of _counts_backward."""
    from . import fp8 as fops

    N, E = dz.shape
    dev = dz.device
    gs32 = dz / lens.clamp(min=1.0)[:, None] if lens is not None else dz
    Np = -(-N // fops.MX_BK) * fops.MX_BK
    g8t, amax_g = fops.quantize_t(gs32, Np)           # (E, Np) e4m3, scale 448 / amax_g
    ct = torch.empty(V, Np, dtype=torch.uint8, device=dev)
    check(lib().pv_transpose_u8(P(C8), C8.stride(0), N, V, P(ct), Np, stream(dev)), "pv_transpose_u8")
    check(lib().pv_gemm_mx8(P(ct), Np, P(g8t), Np, P(out), out.stride(0), V, E, Np, 1, 0, None,
                            1.0 / fops.FP8_MAX, P(amax_g), 0, 0, stream(dev)), "pv_gemm_mx8(wgrad)")


def embedding_bag(ids: torch.Tensor, W: torch.Tensor, W16: Optional[torch.Tensor] = None, pad: int = 0,
                  mean: bool = True, plan: str = "auto", bias: Optional[torch.Tensor] = None,
                  act: str = "none", fp8: bool = False, w8=None) -> torch.Tensor:
    """(N, L) ids -> (N, E): act(sum (or mean) of the rows of W over non-pad tokens + bias).
    ``act`` in {none, relu, tanh}; bias / act are fused into the producing kernel on the GPU.
    ``fp8``: long bags (the counts plan) multiply e4m3 counts by the per-tensor-scaled e4m3
    table on the block-scaled fp8 MFMA (``w8`` = ops.fp8.quantize_t(W) of this step, else
    quantised here); the weight gradient is e4m3 C^T x the per-tensor e4m3 gradient on the same
    MFMA (PAGEVEC_FP8_BWD=1, opt-in), or the exact bf16 C^T G (straight-through, default)."""
    note_rows(W, ids)  # sparse-gradient tables (parallel/sparse_rows.py) record their rows
    if use_hip(ids, W) and act in _BAG_ACT:
        if W16 is None:
            W16 = W.detach().to(torch.bfloat16).contiguous()
        if plan == "auto":
            plan = "gather" if ids.shape[1] <= 256 else "counts"
        if W.shape[1] % 8:
            plan = "counts"
        if fp8 and FP8_BAG and plan == "counts" and W.shape[1] % 4 == 0 and W.shape[0] <= 40960:
            if w8 is None:
                from . import fp8 as fops

                w8 = fops.quantize_t(W, -(-W.shape[0] // fops.MX_BK) * fops.MX_BK)
            return _BagFn.apply(ids, W, W16, pad, mean, plan, bias, act, w8)
        return _BagFn.apply(ids, W, W16, pad, mean, plan, bias, act)
    if fp8 and ids.shape[1] > 256:  # CPU reference of the fp8 bag: e4m3 counts x e4m3 W (STE)
        return _bag_fp8_reference(ids, W, pad, mean, bias, act)
    out = ref.embedding_bag_sum(ids, W, pad)
    if mean:
        out = out / (ids != pad).sum(dim=1, keepdim=True).clamp(min=1).to(out.dtype)
    if bias is not None:
        out = out + bias
    return dops._torch_act(out, act)


class _Fp8BagRef(torch.autograd.Function):
    """CPU reference of the fp8 bag product: forward e4m3(C) @ e4m3(W) (per-tensor scaled);
    backward as the GPU's: with FP8_BWD the e4m3 counts^T times the per-tensor e4m3 quantised
    gradient (_fp8_weight_grad), else the exact C^T G (straight-through)."""

    @staticmethod
    def forward(ctx, C, W):
        from . import fp8 as fops

        ctx.save_for_backward(C)
        return fops.emulate_e4m3(C) @ fops._emulate(W.detach())

    @staticmethod
    def backward(ctx, g):
        from . import fp8 as fops

        C, = ctx.saved_tensors
        if not FP8_BWD:
            return None, C.t() @ g
        amax = float(g.abs().max())
        gq = fops.emulate_e4m3(g * (fops.FP8_MAX / max(amax, 1e-12))) * (max(amax, 1e-12) / fops.FP8_MAX)
        return None, fops.emulate_e4m3(C).t() @ gq


def _bag_fp8_reference(ids, W, pad, mean, bias, act):
    from . import fp8 as fops

    V = W.shape[0]
    valid = (ids != pad) & (ids >= 0) & (ids < V)
    C = torch.zeros(ids.shape[0], V, dtype=torch.float32, device=ids.device)
    C.scatter_add_(1, torch.where(valid, ids, torch.zeros_like(ids)).long(), valid.float())
    lens = valid.sum(dim=1).float()
    if W.requires_grad and torch.is_grad_enabled():
        out = _Fp8BagRef.apply(C, W)
    else:
        with torch.no_grad():
            out = fops.emulate_e4m3(C) @ fops._emulate(W.detach())
    if mean:
        out = out / lens.clamp(min=1.0)[:, None]
    if bias is not None:
        out = out + bias
    return dops._torch_act(out, act)


def trigram_hash(text: torch.Tensor, lens: torch.Tensor, L: int, hash_size: int) -> torch.Tensor:
    """Device letter-trigram hashing of ASCII byte rows (uint8 (N, Lmax)) -> int32 (N, L)."""
    if use_hip(text):
        N, Lmax = text.shape
        out = torch.empty(N, L, dtype=torch.int32, device=text.device)
        check(lib().pv_trigram_hash(P(text.contiguous()), P(lens.to(torch.int32).contiguous()), P(out), N, Lmax, L,
                                    hash_size, stream(text.device)), "pv_trigram_hash")
        return out
    return ref.fnv1a_trigram_ids(text.cpu(), lens.cpu(), L, hash_size).to(text.device)

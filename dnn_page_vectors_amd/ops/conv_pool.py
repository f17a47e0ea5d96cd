"""Fused embedding-gather -> dropout -> Conv1D(3,4) -> max-pool -> ReLU (the CDSSM tower body).

GPU: ``csrc/kernels/conv_pool_fwd.hip`` (forward, MFMA, weights register-resident)
and ``conv_pool_bwd.hip`` + ``radix_sort.hip`` (sparse argmax backward).  CPU:
``ops/reference.py`` (identical semantics incl. the counter-based dropout mask).
``dtype="fp32"`` (reference precision) on the GPU: ``csrc/kernels/conv_pool_f32.hip`` (fp32 MFMA
forward, fp32 sparse backward; ``_ConvPoolF32Fn``).

Reference layers: Embedding -> Dropout(0.25) -> Graph{Convolution1D(150, k, relu) ->
MaxPooling1D(L-k+1) -> Flatten} x k in (3,4) -> concat (dssm_cnn_v2/cnn_dssm_th.py:83-134).
"""
from __future__ import annotations

import os
import threading

from typing import Optional, Tuple

import torch

from . import determinism, grad_sink
from . import reference as ref
from ._common import P, check, lib, need, ref_precision, stream, use_hip
from ..parallel.sparse_rows import note_rows

EP = 104          # padded embedding row stride of the bf16 table copy (kernel constant)
FW = 150          # filters per width the fast kernel is built for
WIDTHS = (3, 4)
SLOTS_PER_SAMPLE = 7 * FW  # dTable entries per sample: 3 per k=3 filter + 4 per k=4 filter


def fast_path_supported(E: int, widths, num_filters: int) -> bool:
    return tuple(widths) == WIDTHS and num_filters == FW and E <= EP


def table_bf16(table: torch.Tensor) -> torch.Tensor:
    """fp32 (V, E) -> bf16 (V, EP) with zero padding (the layout the kernels gather from)."""
    V, E = table.shape
    out = torch.empty(V, EP, dtype=torch.bfloat16, device=table.device)
    check(lib().pv_cast_pad_bf16(P(table.contiguous()), P(out), V, E, EP, stream(table.device)), "pv_cast_pad_bf16")
    return out


def pack_weights(w3: torch.Tensor, w4: torch.Tensor) -> torch.Tensor:
    """(150,3,E), (150,4,E) fp32 -> MFMA B-fragment order bf16 (see pack_conv_weights_kernel)."""
    E = w3.shape[2]
    n = lib().pv_conv_packed_size()
    out = torch.empty(n, dtype=torch.bfloat16, device=w3.device)
    check(lib().pv_conv_pack_weights(P(w3.contiguous()), P(w4.contiguous()), E, P(out), stream(w3.device)),
          "pv_conv_pack_weights")
    return out


PREP_MULTI = True  # A/B switch (tools/step_flag_ab.py --flag PREP_MULTI): one-launch tower prep


def prep_towers(towers) -> list:
    """[(table (V,E), w3, w4), ...] -> [(table_bf16, packed weights), ...] — the per-step compute
    copies of every conv tower in one launch per 4 towers (pv_conv_prep_multi) instead of two per
    tower (table_bf16 + pack_weights)."""
    import ctypes
    out = []
    n_pack = lib().pv_conv_packed_size()
    for g in range(0, len(towers), 4):
        grp = [(t.contiguous(), w3.contiguous(), w4.contiguous()) for t, w3, w4 in towers[g:g + 4]]
        E = grp[0][0].shape[1]
        res = [(torch.empty(t.shape[0], EP, dtype=torch.bfloat16, device=t.device),
                torch.empty(n_pack, dtype=torch.bfloat16, device=t.device)) for t, _, _ in grp]
        n = len(grp)
        arrs = [(ctypes.c_void_p * n)(*[P(x) for x in col]) for col in
                ([t for t, _, _ in grp], [r[0] for r in res], [w for _, w, _ in grp], [w for _, _, w in grp],
                 [r[1] for r in res])]
        Vs = (ctypes.c_int * n)(*[t.shape[0] for t, _, _ in grp])
        check(lib().pv_conv_prep_multi(n, *[ctypes.addressof(a) for a in arrs], ctypes.addressof(Vs), E,
                                       stream(grp[0][0].device)), "pv_conv_prep_multi")
        out.extend(res)
    return out


def _dropout_args(p: float, training: bool, mode: str) -> Tuple[int, int, float]:
    if not training or p <= 0.0 or mode == "none":
        return 0, 0, 1.0
    thr = ref.dropout_threshold(p)
    return thr, 1 if mode == "token" else 0, 256.0 / (256.0 - thr)


_grid_cache = {}

# sorted dTable entries per wave in the reduce (conv_bwd_reduce7_kernel; multiple of 64)
REDUCE_EPW = int(os.environ.get("PAGEVEC_REDUCE_EPW", "512"))


KEYS32 = False  # tests: the 4-byte-key instantiation at a small vocabulary (no env switch)


def _k16(V: int) -> bool:
    """2-byte dTable sort keys (token ids < 65535, sentinel V); 4-byte keys above."""
    return V < 65535 and not KEYS32

# dW/db kernel on a side HIP stream, concurrent with the dTable emit -> sort -> reduce chain
# (both halves are gather/latency-bound and leave CU slots idle when run back to back)
# (round 1: no gain, 9.30 vs 9.30 ms; with the round-2 backward, same box: 7.535 / 7.555 vs
# 7.596 / 7.624 ms per headline step, so it was on).  Round 4, with the sort moved into the
# forward and a side stream per tower, same-process interleaved A/B (tools/step_flag_ab.py,
# profiles/r4_prune/flags_ab.txt): OFF is faster in 15 of 16 rounds on two boxes, 6.848 vs
# 6.869 and 7.266 vs 7.292 ms medians; chunked CDSSM 1.331 vs 1.384 ms; char level (B 1024)
# neutral, 3.587 vs 3.571 — dW after the page tower's reduce on its own stream
DW_SIDE_STREAM = os.environ.get("PAGEVEC_DW_STREAM", "0") != "0"
# conv bias gradients written by the dW kernel straight into the bias parameters' flat-gradient
# slices (0: a zeroed (2 * FW) buffer returned to autograd, AccumulateGrad adds; A/B switch)
BIAS_SINK = os.environ.get("PAGEVEC_BIAS_SINK", "1") != "0"
_side = {}
# one side stream per calling stream (page / query tower) or one shared (A/B)
SIDE_PER_STREAM = os.environ.get("PAGEVEC_SIDE_PER_STREAM", "1") != "0"


def _side_stream(dev: torch.device) -> torch.cuda.Stream:
    """The side stream of the CALLING stream: the page tower (main stream) and the query tower
    (its own stream, models/base.py) each get one, so one tower's dW / early sort never queues
    behind the other's (one shared side stream serialized the two dW kernels: the page dW
    started only after the query dW, and ran alone at the end of the step)."""
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    key = (idx, torch.cuda.current_stream(idx).cuda_stream if SIDE_PER_STREAM else 0)
    if key not in _side and sum(1 for k in _side if k[0] == idx) >= 4:
        key = (idx, 0)  # callers on many streams share one (bounded: no stream per caller stream)
    if key not in _side:
        _side[key] = torch.cuda.Stream(device=idx)
    return _side[key]

# Device seed offset for captured (hipGraph) training steps: when set, every conv kernel
# adds *_SEED_DEV to its seed, so one captured graph draws fresh dropout masks per replay.
_SEED_DEV: Optional[torch.Tensor] = None


def set_seed_tensor(t: Optional[torch.Tensor]) -> None:
    global _SEED_DEV
    _SEED_DEV = t


def _grid(device: torch.device) -> int:
    idx = device.index if device.index is not None else torch.cuda.current_device()
    if idx not in _grid_cache:
        _grid_cache[idx] = torch.cuda.get_device_properties(idx).multi_processor_count
    return _grid_cache[idx]


# dTable sort: the in-tree stable LSD radix sort (radix_sort.hip: graph-safe, no memsets /
# atomics).  The one-pass counting sort (0.435 vs 0.291 ms at 17.2 M keys) and rocPRIM's
# onesweep sort (its memset-reset state faulted under long hipGraph replays) were measured
# and removed: docs/PERF.md "dTable sort".


def sort_pairs_iota(keys: torch.Tensor, skeys: torch.Tensor, svals: torch.Tensor, end_bit: int) -> None:
    """Stable sort of ``keys`` (int16 / int32, read as unsigned) by bits [0, end_bit): sorted
    keys -> ``skeys``, their input positions -> ``svals`` (int32)."""
    L_ = lib()
    M = keys.numel()
    s = stream(keys.device)
    kb = keys.element_size()
    tb = int(L_.pv_rsort_temp_bytes(M, end_bit, kb))
    temp = torch.empty(max(tb, 1), dtype=torch.uint8, device=keys.device)
    check(L_.pv_rsort_pairs(P(temp), tb, P(keys), P(skeys), None, P(svals), M, end_bit, kb, s), "pv_rsort_pairs")


# the dTable sort keys written by the conv FORWARD's loader waves, one sample behind the MFMA
# waves (each filter's argmax window and ReLU liveness are known then): the backward only
# writes the {g * scale, argmax} records instead of running the emit kernel's id gathers on
# its critical path (PAGEVEC_FWD_EMIT=0: the emit kernel)
FWD_EMIT = os.environ.get("PAGEVEC_FWD_EMIT", "1") != "0"
# ... and sorted right after the forward, on the side stream (PAGEVEC_EARLY_SORT=0: in the
# backward, on its critical path)
EARLY_SORT = os.environ.get("PAGEVEC_EARLY_SORT", "1") != "0"
# ... except for mid-length sequences (EARLY_SORT_SKIP_L[0] < L < EARLY_SORT_SKIP_L[1], the
# chunk encoders' 512-token chunks): there the early sort competes with a short forward and the
# loss instead of hiding behind a long page conv.  Same-process A/B (tools/step_flag_ab.py,
# profiles/r4_prune/flags_ab.txt): early sort always on vs only for L >= 1024 — chunked CDSSM
# 1.247 vs 1.148 ms, but the headline 6.764 vs 6.886 (its 45-token query tower gains from it)
# and char level neutral; hence the skip window instead of a threshold.
EARLY_SORT_SKIP = os.environ.get("PAGEVEC_EARLY_SORT_SKIP", "1") != "0"
EARLY_SORT_SKIP_L = (128, 1024)


def _early_sort(L: int) -> bool:
    lo, hi = EARLY_SORT_SKIP_L
    return EARLY_SORT and not (EARLY_SORT_SKIP and lo < L < hi)


V7_DBG = (16384 + 64 + 5 + 1024, 16384 + 64 + 5, 16384 + 128 + 5, 16384 + 128 + 5 + 1024,
          16384 + 192 + 5 + 1024)  # pv_conv_set_dbg variants with the loader key emit (every v7 arm)


def _capture_streams() -> bool:
    """Side streams inside a hipGraph capture (models/base.py CAPTURE_STREAMS) — except a fork
    of a fork: the query tower's early sort (a side stream of the query stream, itself forked
    from the capture stream) made hipStreamEndCapture segfault (round 6: query stream alone and
    early sort alone capture fine, both together crash), so inside a capture the query tower
    sorts in its backward."""
    from ..models.base import CAPTURE_STREAMS, QUERY_STREAM_IDS

    if not CAPTURE_STREAMS:
        return False
    if torch.cuda.is_current_stream_capturing() and torch.cuda.current_stream().cuda_stream in QUERY_STREAM_IDS:
        return False
    return True


def _conv_dbg() -> int:
    return int(lib().pv_conv_get_dbg())


def _weight_rows(w3: torch.Tensor, w4: torch.Tensor, ep: int) -> torch.Tensor:
    """bf16 weight rows [2*FW][4][EP] (zero padded): the operands the forward MFMAs used."""
    F, _, E = w3.shape
    if w3.is_cuda and F == FW and ep == EP and w3.dtype == torch.float32 and w4.dtype == torch.float32:
        wrow = torch.empty(2 * F, 4, ep, dtype=torch.bfloat16, device=w3.device)  # one launch
        check(lib().pv_conv_weight_rows(P(w3.detach().contiguous()), P(w4.detach().contiguous()), E, P(wrow),
                                        stream(w3.device)), "pv_conv_weight_rows")
        return wrow
    wrow = torch.zeros(2 * F, 4, ep, dtype=torch.bfloat16, device=w3.device)
    wrow[:F, :3, :E] = w3.detach()
    wrow[F:, :, :E] = w4.detach()
    return wrow


_CALLER_GRAD = threading.local()  # grad mode at the _ConvPoolFn.apply call site
_CALLER_GRAD.on = True


class _ConvPoolFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, ids, table, w3, w4, b3, b4, tbl16, wpack, p, seed, row_offset, training, mode):
        ids = need(ids, torch.int32, "ids", 2)
        N, L = ids.shape
        V, E = table.shape
        if L < 4:
            raise ValueError("sequence length must be >= 4 for filter widths (3,4)")
        thr, tok, scale = _dropout_args(p, training, mode)
        pooled = torch.empty(N, 2 * FW, dtype=torch.float32, device=ids.device)
        argmax = torch.empty(N, 2 * FW, dtype=torch.int32, device=ids.device)
        seed &= 0xFFFFFFFF
        row_offset &= 0xFFFFFFFF
        sp = _SEED_DEV
        b3c, b4c = b3.detach().contiguous(), b4.detach().contiguous()  # the parameters themselves: no cat
        keys = None
        # needs_input_grad reflects requires_grad, not grad mode, and forward() itself runs with
        # grad disabled: the caller's grad mode (_CALLER_GRAD) says whether a backward can
        # follow.  Under no_grad (eval, Recall / encode batches) no keys are emitted or sorted.
        if _CALLER_GRAD.on and ctx.needs_input_grad[1] and FWD_EMIT and _conv_dbg() in (0,) + V7_DBG:
            k16 = _k16(V)
            keys = torch.empty(N * SLOTS_PER_SAMPLE, dtype=torch.int16 if k16 else torch.int32, device=ids.device)
        check(lib().pv_conv_pool_fwd2(P(ids), P(tbl16), P(wpack), P(b3c), P(b4c), P(pooled), P(argmax), N, L, V,
                                      seed, P(sp), row_offset, thr, tok, scale, _grid(ids.device), stream(ids.device),
                                      P(keys), 0 if keys is None else keys.element_size()),
              "pv_conv_pool_fwd2")
        ctx.keys = keys
        ctx.sorted = None
        if keys is not None and _early_sort(L) and (_capture_streams() or not torch.cuda.is_current_stream_capturing()) \
                and not determinism.enabled():
            # the sort of the table-gradient keys depends on the forward alone: run it now on
            # the side stream, beside the rest of the forward and the loss, instead of on the
            # backward's critical path (the backward waits for its event before the reduce)
            main = torch.cuda.current_stream(ids.device)
            side = _side_stream(ids.device)
            skeys = torch.empty_like(keys)
            svals = torch.empty(keys.numel(), dtype=torch.int32, device=ids.device)
            side.wait_stream(main)
            with torch.cuda.stream(side):
                sort_pairs_iota(keys, skeys, svals, max(1, int(V).bit_length()))
            for t in (keys, skeys, svals):
                t.record_stream(side)
            ev = torch.cuda.Event()
            ev.record(side)
            ctx.sorted = (skeys, svals, ev)
        ctx.save_for_backward(ids, pooled, argmax, tbl16, w3, w4)
        ctx.meta = (V, E, seed, row_offset, thr, tok, scale, sp)
        ctx.mark_non_differentiable(argmax)
        ctx.set_materialize_grads(False)  # no zero-filled (N, 300) int gradient for argmax
        ctx.params = (table, w3, w4, b3, b4)  # flat-gradient direct-write targets (ops/grad_sink.py)
        return pooled, argmax

    @staticmethod
    def backward(ctx, gpool, _gargmax):
        if gpool is None:
            return (None,) * 13
        ids, pooled, argmax, tbl16, w3, w4 = ctx.saved_tensors
        V, E, seed, row_offset, thr, tok, scale, sp = ctx.meta
        N, L = ids.shape
        dev = ids.device
        s = stream(dev)
        gpool = gpool.contiguous().float()
        # the backward kernels accumulate atomically: they can add straight into the flat
        # gradient buffer (no zeroed temporaries, no AccumulateGrad adds)
        ptable, pw3, pw4, pb3, pb4 = ctx.params
        t_tab = grad_sink.accum_target(ptable) if ctx.needs_input_grad[1] else None
        t3 = grad_sink.accum_target(pw3) if ctx.needs_input_grad[2] else None
        t4 = grad_sink.accum_target(pw4) if ctx.needs_input_grad[3] else None
        tb3 = grad_sink.accum_target(pb3) if ctx.needs_input_grad[4] and BIAS_SINK else None
        tb4 = grad_sink.accum_target(pb4) if ctx.needs_input_grad[5] and BIAS_SINK else None
        dw3 = t3 if t3 is not None else torch.zeros_like(w3)
        dw4 = t4 if t4 is not None else torch.zeros_like(w4)
        db = None
        if tb3 is None or tb4 is None:
            db = torch.zeros(2 * FW, dtype=torch.float32, device=dev)
        db3 = tb3 if tb3 is not None else db[:FW]
        db4 = tb4 if tb4 is not None else db[FW:]
        L_ = lib()
        # every buffer the side stream touches is allocated on the main stream above/before
        # and the main stream joins the side stream before returning: no cross-stream reuse
        # the page tower's dW beside its table chain (not inside a hipGraph capture: one stream)
        side = (_side_stream(dev) if DW_SIDE_STREAM and ctx.needs_input_grad[1]
                and (_capture_streams() or not torch.cuda.is_current_stream_capturing()) and not determinism.enabled()
                else None)
        if side is not None:
            main = torch.cuda.current_stream(dev)
            side.wait_stream(main)
            s_dw = side.cuda_stream

        def launch_dw():
            check(L_.pv_conv_pool_bwd_dw2(P(gpool), P(pooled), P(argmax), P(ids), P(tbl16), P(dw3), P(dw4), P(db3),
                                          P(db4), N, L, E, V, seed, P(sp), row_offset, thr, tok, scale,
                                          s_dw if side is not None else s), "pv_conv_pool_bwd_dw2")

        # Order: the side-stream variant starts dW first (it runs beside the table chain);
        # on one stream the TABLE gradient goes first.  Either way the table's data-parallel
        # bucket (a bucket of its own, parallel/ddp.py) is released as soon as its reduce is
        # enqueued on this stream, so its all-reduce (12 MB for the 30k x 100 table) overlaps
        # the dW kernel instead of trailing the whole backward.
        if side is not None:
            launch_dw()
        dtable = None
        if ctx.needs_input_grad[1]:
            M = N * SLOTS_PER_SAMPLE  # k3 filters 3 slots, k4 filters 4 (conv_bwd_emit3_kernel)
            u32 = torch.int32
            end_bit = max(1, int(V).bit_length())
            rec = torch.empty(N * 2 * FW, 2, dtype=torch.int32, device=dev)  # {g * scale, argmax}
            # entry i's value is its slot i: no value array, the sort reads a counting iterator;
            # token ids < 65535 sort as 2-byte keys
            k16 = _k16(V)
            keys, ctx.keys = ctx.keys, None
            early, ctx.sorted = ctx.sorted, None
            if early is not None:  # keys written and sorted during the forward
                skeys, svals, ev = early
            else:
                skeys = torch.empty(M, dtype=torch.int16 if k16 else u32, device=dev)
                svals = torch.empty(M, dtype=u32, device=dev)
            if keys is not None:  # written by the forward: only the records remain
                check(L_.pv_conv_pool_bwd_rec(P(gpool), P(argmax), P(rec), N, scale, s), "pv_conv_pool_bwd_rec")
            elif k16:
                keys = torch.empty(M, dtype=torch.int16, device=dev)
                check(L_.pv_conv_pool_bwd_emit3_u16(P(gpool), P(pooled), P(argmax), P(ids), P(keys), P(rec), N, L, V,
                                                    scale, s), "pv_conv_pool_bwd_emit3_u16")
            else:
                keys = torch.empty(M, dtype=u32, device=dev)
                check(L_.pv_conv_pool_bwd_emit3(P(gpool), P(pooled), P(argmax), P(ids), P(keys), None, P(rec), N, L,
                                                V, scale, s), "pv_conv_pool_bwd_emit3")
            if early is not None:
                torch.cuda.current_stream(dev).wait_event(ev)
            else:
                sort_pairs_iota(keys, skeys, svals, end_bit)
            dtable = t_tab if t_tab is not None else torch.zeros(V, E, dtype=torch.float32, device=dev)
            wrow = _weight_rows(w3, w4, EP)
            fn = "pv_conv_pool_bwd_reduce7_u16" if k16 else "pv_conv_pool_bwd_reduce7"
            check(getattr(L_, fn)(P(skeys), P(svals), P(rec), P(wrow), P(dtable), M, REDUCE_EPW, L, E, V, seed, P(sp),
                                  row_offset, thr, tok, s), fn)
        if t_tab is not None:
            grad_sink.done(ptable)  # fires the table's bucket: enqueued after the reduce above
        if side is None:
            launch_dw()
        else:
            main.wait_stream(side)
        for t, prm in ((t3, pw3), (t4, pw4), (tb3, pb3), (tb4, pb4)):
            if t is not None:
                grad_sink.done(prm)
        if t_tab is not None:
            dtable = None
        return (None, dtable, None if t3 is not None else dw3, None if t4 is not None else dw4,
                None if tb3 is not None else db3, None if tb4 is not None else db4,
                None, None, None, None, None, None, None)


# ---- reference precision (dtype="fp32"): csrc/kernels/conv_pool_f32.hip -------------------
F32_EMAX = 112  # conv_pool_f32.hip EMAX (LDS sizing)
# 0: the fp32 dTable always uses global row atomics (A/B of the LDS-privatised small-V path)
F32_DX_LDS = os.environ.get("PAGEVEC_F32_DX_LDS", "1") != "0"
# 0: the fp32 kernels recompute the dropout hashes instead of reading the keep-bit plane (A/B)
F32_MASK = os.environ.get("PAGEVEC_F32_MASK", "1") != "0"


def f32_supported(E: int, widths, num_filters: int) -> bool:
    return tuple(widths) == WIDTHS and num_filters == FW and E % 4 == 0 and 4 <= E <= F32_EMAX


def f32_plan(N: int, L: int, n_cu: int) -> Tuple[int, int, int]:
    """(nslots, nseg, sw) of the fp32 forward: nslots persistent workgroups per filter group
    (5 groups, one workgroup per CU: 159 KB of LDS), each sample's L - 2 windows cut into nseg
    segments of sw windows (a multiple of the 128-window chunk) so that every group has >= 32
    (sample, segment) items per workgroup (tail imbalance <= 3 %)."""
    cw, ng = 128, 5
    nslots = max(1, n_cu // ng)
    nch = -(-(L - 2) // cw)
    nseg = max(1, min(nch, -(-32 * nslots // max(N, 1))))
    sw = -(-nch // nseg) * cw
    nseg = -(-(L - 2) // sw)
    return max(1, min(nslots, N * nseg)), nseg, sw


F32_DXW_MAX = 10240  # conv_pool_f32.hip DXW_MAX: wave-private tables (deterministic sums)


def _f32_dtable_ordered(gpool, pooled, argmax, ids, w3, w4, dtable, seed, row_offset, thr, tok, scale):
    """dTable += scale * g[n, f] * W[f, j, :] * keep(n, a + j, :) at row ids[n, a + j] for every live
    (n, f) pair, accumulated by torch's deterministic index_add_ (determinism mode)."""
    N, L = ids.shape
    V, E = dtable.shape
    live = (pooled > 0) & (gpool != 0)
    n_i, f_i = live.nonzero(as_tuple=True)
    a = argmax[n_i, f_i].long()
    g = gpool[n_i, f_i] * scale
    for W, K, lo, hi in ((w3, 3, 0, FW), (w4, 4, FW, 2 * FW)):
        sel = (f_i >= lo) & (f_i < hi)
        n_, f_, a_, g_ = n_i[sel], f_i[sel] - lo, a[sel], g[sel]
        t = a_[:, None] + torch.arange(K, device=ids.device)
        tk = ids[n_[:, None], t].long()
        contrib = g_[:, None, None] * W[f_]
        if thr > 0:
            keep = ref.dropout_keep_mask(seed, 0, E, thr / 256.0, row_offset, "token" if tok else "element",
                                         rows=n_[:, None] * L + t)
            contrib = contrib * keep.view(-1, K, E).to(contrib.dtype)
        ok = (tk >= 0) & (tk < V)
        dtable.index_add_(0, tk[ok], contrib[ok])


class _ConvPoolF32Fn(torch.autograd.Function):
    """fp32 gather -> dropout -> conv(3, 4) -> max-pool -> ReLU with fp32 MFMAs, and its sparse
    argmax backward (dW / db per-split partials summed in order; dTable fp32 row atomics)."""

    @staticmethod
    def forward(ctx, ids, table, w3, w4, b3, b4, p, seed, row_offset, training, mode):
        ids = need(ids, torch.int32, "ids", 2)
        N, L = ids.shape
        V, E = table.shape
        if L < 4:
            raise ValueError("sequence length must be >= 4 for filter widths (3,4)")
        thr, tok, scale = _dropout_args(p, training, mode)
        tab = table.detach().contiguous()
        w3c, w4c = w3.detach().contiguous(), w4.detach().contiguous()
        nslots, nseg, sw = f32_plan(N, L, _grid(ids.device))
        part = torch.empty(N * nseg, 2 * FW, 2, dtype=torch.float32, device=ids.device)
        pooled = torch.empty(N, 2 * FW, dtype=torch.float32, device=ids.device)
        argmax = torch.empty(N, 2 * FW, dtype=torch.int32, device=ids.device)
        seed &= 0xFFFFFFFF
        row_offset &= 0xFFFFFFFF
        sp = _SEED_DEV
        # dropout keep bits, one u32 per 32 columns per row, shared by the forward's five filter
        # groups (instead of each recomputing the hashes)
        wpr = (E + 31) // 32
        mask = None
        if thr > 0 and F32_MASK:
            mask = torch.empty(N * L * wpr, dtype=torch.int32, device=ids.device)
            check(lib().pv_conv_f32_mask(P(mask), N * L, wpr, seed, P(sp), row_offset, thr, tok, stream(ids.device)),
                  "pv_conv_f32_mask")
        check(lib().pv_conv_f32_fwd(P(ids), P(tab), P(w3c), P(w4c), P(b3.detach().contiguous()),
                                    P(b4.detach().contiguous()), P(part), P(pooled), P(argmax), N, L, V, E, nseg, sw,
                                    nslots, seed, P(sp), row_offset, thr, tok, scale, P(mask), wpr,
                                    stream(ids.device)),
              "pv_conv_f32_fwd")
        ctx.save_for_backward(ids, tab, w3c, w4c, pooled, argmax)
        # the backward kernels recompute the hashes: they are latency-bound on their gathers, and
        # a dependent mask-word load cost more than the VALU (dx 0.58 -> 0.74, dW 0.17 -> 0.30 ms
        # per step with the plane)
        ctx.mask = None
        ctx.meta = (V, E, seed, row_offset, thr, tok, scale, sp, wpr)
        ctx.mark_non_differentiable(argmax)
        ctx.set_materialize_grads(False)
        return pooled, argmax

    @staticmethod
    def backward(ctx, gpool, _gargmax):
        if gpool is None:
            return (None,) * 11
        ids, tab, w3, w4, pooled, argmax = ctx.saved_tensors
        V, E, seed, row_offset, thr, tok, scale, sp, wpr = ctx.meta
        mask, ctx.mask = ctx.mask, None
        N, L = ids.shape
        dev = ids.device
        s = stream(dev)
        gpool = gpool.contiguous().float()
        dtable = None
        if ctx.needs_input_grad[1] and determinism.enabled() and V * E > F32_DXW_MAX:
            # deterministic mode: the LDS / global float-atomic table kernels sum in arrival
            # order; torch's deterministic index_add_ over the (pair, row) contributions instead
            dtable = torch.zeros(V, E, dtype=torch.float32, device=dev)
            _f32_dtable_ordered(gpool, pooled, argmax, ids, w3, w4, dtable, seed, row_offset, thr, tok, scale)
        elif ctx.needs_input_grad[1]:
            dtable = torch.zeros(V, E, dtype=torch.float32, device=dev)
            if V * E <= lib().pv_conv_f32_dx_lds_max() and E <= 128 and F32_DX_LDS:
                # small (char-level) vocabularies: per-workgroup LDS tables, summed in order
                nparts = max(1, min(_grid(dev), -(-N * 2 * FW // 256)))  # one workgroup per CU at most
                partial = torch.empty(nparts, V, E, dtype=torch.float32, device=dev)
                check(lib().pv_conv_f32_bwd_dx_lds(P(gpool), P(pooled), P(argmax), P(ids), P(w3), P(w4), P(partial),
                                                   P(dtable), N, L, E, V, nparts, seed, P(sp), row_offset, thr, tok,
                                                   scale, P(mask), wpr, s), "pv_conv_f32_bwd_dx_lds")
            else:
                check(lib().pv_conv_f32_bwd_dx(P(gpool), P(pooled), P(argmax), P(ids), P(w3), P(w4), P(dtable), N, L,
                                               E, V, seed, P(sp), row_offset, thr, tok, scale, P(mask), wpr, s),
                      "pv_conv_f32_bwd_dx")
        dw3 = dw4 = db3 = db4 = None
        if any(ctx.needs_input_grad[2:6]):
            nsplit = max(1, min(128, N // 16))  # 16 samples per (filter, split) block: 4 per wave
            dwpart = torch.empty(nsplit, 2 * FW, 4 * E, dtype=torch.float32, device=dev)
            dbpart = torch.empty(nsplit, 2 * FW, dtype=torch.float32, device=dev)
            check(lib().pv_conv_f32_bwd_dw(P(gpool), P(pooled), P(argmax), P(ids), P(tab), P(dwpart), P(dbpart), N,
                                           L, E, V, nsplit, seed, P(sp), row_offset, thr, tok, scale, P(mask), wpr,
                                           s),
                  "pv_conv_f32_bwd_dw")
            dw3 = dwpart[:, :FW, :3 * E].sum(0).view(FW, 3, E)
            dw4 = dwpart[:, FW:, :].sum(0).view(FW, 4, E)
            db = dbpart.sum(0)
            db3, db4 = db[:FW], db[FW:]
        return (None, dtable, dw3, dw4, db3, db4, None, None, None, None, None)


def conv_relu_maxpool_fused(ids: torch.Tensor, table: torch.Tensor, weights, biases, p: float, seed: int,
                            training: bool, mode: str = "element", row_offset: int = 0,
                            compute_cache=None) -> Tuple[torch.Tensor, torch.Tensor]:
    """pooled (N, sum F) post-ReLU, argmax (N, sum F) for one tower invocation.

    ``compute_cache``: optional (tbl16, wpack) already derived from the current params.
    """
    note_rows(table, ids)  # sparse-gradient tables (parallel/sparse_rows.py) record their rows
    if ids.is_cuda and ref_precision() and table.dtype == torch.float32 and \
            f32_supported(table.shape[1], [w.shape[1] for w in weights], weights[0].shape[0]):
        (w3, w4), (b3, b4) = weights, biases
        return _ConvPoolF32Fn.apply(ids, table, w3, w4, b3, b4, float(p), int(seed), int(row_offset), bool(training),
                                    mode)
    if use_hip(ids, table) and fast_path_supported(table.shape[1], [w.shape[1] for w in weights], weights[0].shape[0]):
        w3, w4 = weights
        b3, b4 = biases
        if compute_cache is None:
            tbl16, wpack = table_bf16(table.detach()), pack_weights(w3.detach(), w4.detach())
        else:
            tbl16, wpack = compute_cache
        _CALLER_GRAD.on = torch.is_grad_enabled()
        return _ConvPoolFn.apply(ids, table, w3, w4, b3, b4, tbl16, wpack, float(p), int(seed), int(row_offset),
                                 bool(training), mode)
    if ids.is_cuda and use_hip(ids, table):
        # no silent eager fallback on the GPU: the fused kernel is built for this geometry only
        raise NotImplementedError(
            f"fused CDSSM conv kernel supports filter_sizes={WIDTHS}, num_filters={FW}, embedding_dim<={EP}; got "
            f"filter_sizes={tuple(w.shape[1] for w in weights)}, num_filters={weights[0].shape[0]}, "
            f"embedding_dim={table.shape[1]}. Use dtype='fp32' (reference precision; PyTorch ops for other geometries) "
            f"or the supported geometry.")
    x = ref.embed_dropout(ids, table, p, seed, training, mode) if row_offset == 0 else \
        _embed_dropout_offset(ids, table, p, seed, training, mode, row_offset)
    return ref.conv_relu_maxpool(x, weights, biases)


def _embed_dropout_offset(ids, table, p, seed, training, mode, row_offset):
    x = torch.nn.functional.embedding(ids.long(), table)
    if training and p > 0.0 and mode != "none":
        N, L, E = x.shape
        keep = ref.dropout_keep_mask(seed, N * L, E, p, row_offset=row_offset, mode=mode, device=ids.device)
        x = x * keep.view(N, L, E).to(x.dtype) * (256.0 / (256.0 - ref.dropout_threshold(p)))
    return x

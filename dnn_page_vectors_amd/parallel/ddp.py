"""Bucketed, backward-overlapped gradient all-reduce over the flat gradient buffer.

Data parallelism: every rank holds a full replica; gradients live in one
flat fp32 buffer (ops/optim.FlatParams), cut into contiguous buckets in *reverse*
parameter order (the order autograd produces them).  A post-accumulate-grad hook
counts arrivals per bucket and launches an async all-reduce as soon as a bucket is
complete, so communication of late layers overlaps the backward of early ones.

Bucket size: xGMI is point-to-point (7 links x ~153 GB/s per MI355X); RCCL spreads a
ring/tree over several channels, and messages of a few tens of MB keep them busy while
staying latency-light.  Default 32 MB (the BERT-base gradient, ~440 MB, is ~14 buckets
overlapped with backward).  Buckets are also cut where the top-level module changes
(``query_tower`` | ``doc_towers``): the query tower runs last in forward, so its gradient
(12.6 MB for CDSSM-ngram) is complete early in backward and its all-reduce overlaps the
doc tower's backward instead of sharing one 25 MB bucket launched after everything.
The cut is made at EVERY such boundary, whatever the open bucket's size, so a bucket never
mixes the two towers' parameters.

Streams: the towers' backward passes run on different HIP streams (the query tower on its
side stream, models/base.py; the page tower's dW on the conv side stream, ops/conv_pool.py),
and a bucket's all-reduce is launched from whichever gradient hook completes it.  Every hook
therefore records the stream that was current when its gradient was produced, and
``_launch`` makes the launching stream wait on each of the bucket's producer streams before
it enqueues the collective — the all-reduce can never read a gradient still being written on
another stream, independent of how the buckets are cut.
"""
from __future__ import annotations

from typing import List, Optional

import torch
import torch.distributed as dist

from ..ops import grad_sink
from ..ops.optim import FlatParams
from .dist import active


class GradBuckets:
    MIN_SPLIT_BYTES = 1 << 20  # embedding tables of at least 1 MB get a bucket of their own
    OWN_BUCKET_LEAVES = ("embedding", "word")  # >= 1 MB embedding tables: one bucket each

    def __init__(self, flat: FlatParams, bucket_mb: float = 32.0, overlap: bool = True, reduce: str = "avg",
                 sparse=None):
        """reduce: "avg" (data parallel) or "sum" (tower placement: per-rank partial gradients).
        sparse: parallel/sparse_rows.SparseTables — its tables get a bucket of their own whose
        "all-reduce" is the touched-row exchange (averaged like the dense buckets)."""
        self.flat = flat
        self.bucket_mb = float(bucket_mb)
        self.sparse = sparse
        if sparse is not None and reduce == "sum":
            raise ValueError("sparse gradient tables average over ranks (data parallel), not tower placement")
        self.sparse_bucket = {}
        self.world = dist.get_world_size() if dist.is_initialized() else 1
        self.active = active()  # world > 1, or the forced one-rank rehearsal (PAGEVEC_FORCE_DIST)
        self.overlap = overlap and self.active
        self.sum_only = reduce == "sum"
        self.avg_op = None
        if self.active and not self.sum_only:
            self.avg_op = dist.ReduceOp.AVG if dist.get_backend() == "nccl" else None
        cap = max(1, int(bucket_mb * (1 << 20) / 4))
        self.buckets: List[List[int]] = []  # [lo, hi, n_params]
        self.param_bucket = {}
        cur_lo = cur_hi = None
        cur_mod = None
        members: List[str] = []
        min_split = self.MIN_SPLIT_BYTES // 4
        for name, p in reversed(flat.named):
            o, k, _ = flat.offsets[name]
            end = o + (k + 63) // 64 * 64
            mod = name.split(".", 1)[0]
            own = name.rsplit(".", 1)[-1] in self.OWN_BUCKET_LEAVES and (end - o) >= min_split
            if sparse is not None and name in sparse.tables:
                own = True
            if own:
                # embedding tables get a bucket of their own: the sparse table backward
                # releases it before the tower's weight gradients are done (ops/conv_pool.py)
                if cur_lo is not None:
                    self._add(cur_lo, cur_hi, members)
                self._add(o, end, [name])
                if sparse is not None and name in sparse.tables:
                    self.sparse_bucket[len(self.buckets) - 1] = sparse.tables[name]
                cur_lo = cur_hi = cur_mod = None
                members = []
                continue
            if cur_lo is None:
                cur_lo, cur_hi, members, cur_mod = o, end, [name], mod
            elif mod != cur_mod:  # never mix towers in one bucket
                self._add(cur_lo, cur_hi, members)
                cur_lo, cur_hi, members, cur_mod = o, end, [name], mod
            elif (cur_hi - o) <= cap:
                cur_lo = o
                members.append(name)
            else:
                self._add(cur_lo, cur_hi, members)
                cur_lo, cur_hi, members, cur_mod = o, end, [name], mod
        if cur_lo is not None:
            self._add(cur_lo, cur_hi, members)
        self.pending: List[set] = [set() for _ in self.buckets]
        self.streams: List[dict] = [{} for _ in self.buckets]  # producer streams per bucket
        self.handles: List[Optional[object]] = [None] * len(self.buckets)
        self._hooks = []
        if self.overlap:
            for name, p in flat.named:
                bi = self.param_bucket[name]
                hook = self._make_hook(bi)
                self._hooks.append(p.register_post_accumulate_grad_hook(hook))
                # ops that write the flat gradient directly fire this instead (ops/grad_sink.py)
                self._hooks.append(_Remover(grad_sink.add_hook(p, hook)))

    def _add(self, lo: int, hi: int, members: List[str]) -> None:
        bi = len(self.buckets)
        self.buckets.append([lo, hi, len(members)])
        for m in members:
            self.param_bucket[m] = bi

    def _make_hook(self, bi: int):
        def hook(p):
            seen = self.pending[bi]
            seen.add(id(p))  # a set: a parameter reached twice counts once
            if p.is_cuda:
                st = torch.cuda.current_stream(p.device)
                self.streams[bi][st.cuda_stream] = st
            if len(seen) == self.buckets[bi][2] and self.handles[bi] is None:
                self._launch(bi)
        return hook

    def _launch(self, bi: int) -> None:
        lo, hi, _ = self.buckets[bi]
        view = self.flat.grad[lo:hi]
        t = self.sparse_bucket.get(bi)
        if view.is_cuda:  # order the collective after every stream that wrote into the bucket
            cur = torch.cuda.current_stream(view.device)
            for key, st in self.streams[bi].items():
                if key != cur.cuda_stream:
                    cur.wait_stream(st)
        if t is not None:  # touched-row exchange instead of the dense all-reduce
            self.sparse.launch(t)
            self.handles[bi] = "sparse"
            return
        if self.avg_op is not None:
            self.handles[bi] = dist.all_reduce(view, op=self.avg_op, async_op=True)
        else:
            self.handles[bi] = dist.all_reduce(view, op=dist.ReduceOp.SUM, async_op=True)

    def start_step(self) -> None:
        self.pending = [set() for _ in self.buckets]
        self.streams = [{} for _ in self.buckets]
        self.handles = [None] * len(self.buckets)

    def finish(self) -> None:
        """Launch the buckets that never completed (unused params) and wait for all."""
        if not self.active:
            return
        for bi in range(len(self.buckets)):
            if self.handles[bi] is None:
                self._launch(bi)
        for bi, h in enumerate(self.handles):
            if bi in self.sparse_bucket:
                self.sparse.complete(self.sparse_bucket[bi])
                continue
            h.wait()
            if self.avg_op is None and not self.sum_only:
                lo, hi, _ = self.buckets[bi]
                self.flat.grad[lo:hi].div_(self.world)
        self.handles = [None] * len(self.buckets)

    def remove(self) -> None:
        for h in self._hooks:
            h.remove()
        self._hooks = []


class _Remover:
    def __init__(self, fn):
        self.remove = fn


def broadcast_params(flat: FlatParams, src: int = 0) -> None:
    if active():
        dist.broadcast(flat.data, src)

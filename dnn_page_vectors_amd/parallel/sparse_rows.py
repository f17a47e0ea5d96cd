"""Row-sparse gradients for large embedding tables ("for the 7.5 M-word vocab,
all-gather (ids, rows) pairs of the touched rows instead of all-reducing 3 GB").

The reference's word-level v1 loads a 7,556,273-row table (dssm_cnn/data_helpers.py:143)
into ``Embedding(weights=...)`` (dssm_cnn_v2/cnn_dssm_th.py:114-120).  A step touches only
the rows of the tokens in its batch, yet the dense path of this framework would, per table
and step: zero-fill the whole table gradient (3 GB), scan it for the gradient norm and the
non-finite guard, all-reduce it (3 GB over xGMI, ~40 ms per step at W = 8) and run the
optimizer over it.  With ``Configuration.sparse_embedding_grad`` every >= 2-D embedding
table registered here instead:

* the ops that gather its rows (the fused conv tower, the embedding bag, the LSTM's
  F.embedding) ``note`` the token ids of the step; the candidate rows are their union
  (sorted unique ids, one device sort);
* only the previous step's rows are zeroed (the rest of the table gradient stays zero by
  construction), ``FlatParams.zero_grad`` skips the table;
* data parallel: in place of the table's dense bucket all-reduce, every rank all-gathers
  (row ids, gradient rows) padded to a capacity every rank agrees on, zeroes its own rows
  and index-adds everyone's rows scaled by 1/W — the average, exactly what the dense
  all-reduce would have left in those rows, every other row being zero on every rank;
* the optimizer runs LazyAdam over the union rows only (``pv_adam_rows``: the lazy kernel
  over a row list, rows whose gradient is all zero keep weights and moments — the
  ``lazy_embedding_adam`` semantics, so a sparse run equals a lazy dense run);
* the gradient norm / non-finite check reads the union rows, not the table.

Cost per step: O(touched rows x E) instead of O(V x E).

Row lists are FIXED-SIZE device tensors (sorted unique rows, then -1 padding): the union is a
sort + first-of-run flags + a scatter to the run's rank, never ``torch.unique`` or a boolean
mask (both size their output on the host).  ``Configuration.sparse_rows_capacity`` picks the
exchange's padding: -1 (default) = min(V, the largest rank's noted-id count), agreed by one
MAX all-reduce the first time a table is exchanged — no host sync afterwards, so the step is
capturable in a hipGraph; 0 = the exact per-step maximum of distinct rows (a host sync per
table and step: the smallest exchange, not capturable); > 0 = that many rows.  A step whose
distinct rows exceed the capacity counts into ``overflow`` (device); ``check()`` raises on it
(the trainer calls it where it reads metrics anyway).  The Adam row kernel and the gradient
statistics skip -1 entries.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist

from .dist import active


@dataclass
class _Table:
    name: str
    param: torch.nn.Parameter
    off: int
    V: int
    E: int
    notes: List[torch.Tensor] = field(default_factory=list)
    rows: Optional[torch.Tensor] = None      # int32 candidate rows of the current step (after exchange)
    prev: Optional[torch.Tensor] = None      # rows written last step (zeroed before the next)
    pending: Optional[Tuple] = None          # in-flight all-gathers
    prev_buf: Optional[torch.Tensor] = None  # persistent copy of ``prev`` (stable address under capture)
    cap: int = 0                             # agreed exchange capacity (rows), 0 = not yet agreed
    cap_basis: int = 0                       # this rank's noted-id count the capacity was agreed for


def unique_rows(ids: torch.Tensor, V: int, cap: int,
                overflow: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Sorted distinct ids in [0, V) of ``ids`` in a fixed-size int32 tensor of ``cap`` entries,
    padded with -1 — without a host sync.  Distinct ids beyond ``cap`` are dropped and counted
    into ``overflow`` (int64 device scalar) when given."""
    dev = ids.device
    if ids.numel() == 0 or cap <= 0:
        return torch.full((max(cap, 0),), -1, dtype=torch.int32, device=dev)
    x = ids.reshape(-1).to(torch.int64)
    x = torch.where((x >= 0) & (x < V), x, torch.full_like(x, V))  # invalid -> V (sorts last)
    s, _ = torch.sort(x)
    first = torch.ones_like(s, dtype=torch.bool)
    first[1:] = s[1:] != s[:-1]
    first &= s < V
    pos = torch.cumsum(first, 0) - 1
    keep = first & (pos < cap)
    out = torch.full((cap + 1,), -1, dtype=torch.int32, device=dev)
    out.scatter_(0, torch.where(keep, pos, torch.full_like(pos, cap)), torch.where(keep, s, -1).to(torch.int32))
    if overflow is not None:
        overflow += (first & ~keep).sum()
    return out[:cap]


class SparseTables:
    def __init__(self, flat, names: Sequence[str], capacity: int = -1):
        self.flat = flat
        self.capacity = int(capacity)
        self.overflow = torch.zeros((), dtype=torch.int64, device=flat.grad.device)
        named = dict(flat.named)
        self.tables: Dict[str, _Table] = {}
        self._by_id: Dict[int, _Table] = {}
        for n in names:
            o, k, shp = flat.offsets[n]
            if len(shp) != 2:
                raise ValueError(f"sparse gradient table {n!r} must be 2-D, got {tuple(shp)}")
            if shp[1] % 4 or shp[1] > 1024:
                raise ValueError(f"sparse gradient table {n!r}: row length {shp[1]} must be a multiple of 4, <= 1024")
            t = _Table(n, named[n], o, int(shp[0]), int(shp[1]))
            self.tables[n] = t
            self._by_id[id(t.param)] = t
            t.param._pv_sparse = self

    # ---------------------------------------------------------------- per step
    def ranges(self) -> List[Tuple[int, int]]:
        return sorted((t.off, t.off + t.V * t.E) for t in self.tables.values())

    def begin_step(self) -> None:
        """Before the forward: zero the rows written last step (the dense zero skips tables)."""
        for t in self.tables.values():
            if t.prev is not None and t.prev.numel():
                # -1 padding -> row 0: every untouched row of the table gradient is zero
                self.grad2d(t).index_fill_(0, t.prev.clamp(min=0).long(), 0.0)
            t.prev = None
            t.rows = None
            t.notes = []
            t.pending = None

    def note(self, p: torch.Tensor, ids: torch.Tensor) -> None:
        t = self._by_id.get(id(p))
        if t is not None and torch.is_grad_enabled() and p.requires_grad:
            t.notes.append(ids.detach().reshape(-1))

    def grad2d(self, t: _Table) -> torch.Tensor:
        return self.flat.grad[t.off:t.off + t.V * t.E].view(t.V, t.E)

    def _noted(self, t: _Table) -> torch.Tensor:
        if not t.notes:
            return torch.empty(0, dtype=torch.int64, device=self.flat.grad.device)
        return torch.cat([x.to(torch.int64) for x in t.notes]) if len(t.notes) > 1 else t.notes[0]

    def _local_rows(self, t: _Table) -> torch.Tensor:
        ids = self._noted(t)
        return unique_rows(ids, t.V, min(t.V, ids.numel()), self.overflow)

    def _agree_cap(self, t: _Table, ids: torch.Tensor, group) -> int:
        if self.capacity > 0:
            return min(t.V, self.capacity)
        if self.capacity == 0:  # exact: this step's largest distinct-row count (host sync)
            u = unique_rows(ids, t.V, min(t.V, ids.numel()))
            cnt = (u >= 0).sum().reshape(1)
            dist.all_reduce(cnt, op=dist.ReduceOp.MAX, group=group)
            return max(1, int(cnt.item()))
        # auto: agreed from the noted-id counts (host-known shapes) — once, and again whenever a
        # step notes more ids than the count the capacity was agreed for (a larger batch shape),
        # so a later, larger step does not overflow a capacity sized for the first
        n_ids = min(t.V, ids.numel())
        if t.cap == 0 or n_ids > t.cap_basis:
            cnt = torch.tensor([n_ids], dtype=torch.int64, device=ids.device)
            dist.all_reduce(cnt, op=dist.ReduceOp.MAX, group=group)
            t.cap = max(t.cap, 1, int(cnt.item()))
            t.cap_basis = max(t.cap_basis, n_ids)
        return t.cap

    def launch(self, t: _Table, group=None) -> None:
        """The table's gradient is complete: start its row exchange (or just fix its rows)."""
        ids = self._noted(t)
        t.notes = []
        if not active(group):
            t.rows = unique_rows(ids, t.V, min(t.V, ids.numel()), self.overflow)
            return
        W = dist.get_world_size(group)
        cap = self._agree_cap(t, ids, group)
        rows = unique_rows(ids, t.V, cap, self.overflow)
        g2 = self.grad2d(t)
        ok = (rows >= 0).unsqueeze(1)
        vals = torch.where(ok, g2.index_select(0, rows.clamp(min=0).long()), torch.zeros((), dtype=g2.dtype,
                                                                                       device=g2.device))
        all_rows = torch.empty(W * cap, dtype=torch.int32, device=rows.device)
        all_vals = torch.empty(W * cap, t.E, dtype=g2.dtype, device=g2.device)
        h1 = dist.all_gather_into_tensor(all_rows, rows, group=group, async_op=True)
        h2 = dist.all_gather_into_tensor(all_vals, vals, group=group, async_op=True)
        t.pending = (rows, all_rows, all_vals, h1, h2, W)

    def complete(self, t: _Table) -> None:
        """Wait for the exchange; the table gradient rows := the mean over ranks."""
        if t.pending is None:
            return
        u, all_rows, all_vals, h1, h2, W = t.pending
        t.pending = None
        h1.wait()
        h2.wait()
        g2 = self.grad2d(t)
        if g2.is_cuda:
            # launch() ran on the stream of the table's gradient hook (the query tower's side
            # stream when that tower owns the table): these blocks belong to that stream's
            # allocator pool, and without this the next step's side-stream allocations could
            # reuse them before the index_fill_ / index_add_ below have run on this stream
            cur = torch.cuda.current_stream(g2.device)
            for x in (u, all_rows, all_vals):
                x.record_stream(cur)
        # padding entries name row 0 with zero values: zeroing / adding zero to an untouched
        # row (zero by construction) changes nothing
        g2.index_fill_(0, u.clamp(min=0).long(), 0.0)
        g2.index_add_(0, all_rows.clamp(min=0).long(), all_vals, alpha=1.0 / W)
        t.rows = unique_rows(all_rows, t.V, min(t.V, all_rows.numel()))

    def finish_step(self) -> None:
        """After the optimizer: the rows written this step are the next step's zero list."""
        for t in self.tables.values():
            r = t.rows
            if r is not None and (t.prev_buf is None or t.prev_buf.shape != r.shape):
                t.prev_buf = torch.empty_like(r)
            if r is not None:  # a copy at a fixed address: a captured step reads the last replay's
                t.prev_buf.copy_(r)
            t.prev = t.prev_buf if r is not None else None

    def check(self) -> None:
        """Raise if a step's distinct rows ever exceeded the exchange capacity (a host read)."""
        n = int(self.overflow.item())
        if n:
            raise RuntimeError(f"sparse embedding gradients: {n} distinct rows beyond the exchange capacity were "
                               f"dropped (sparse_rows_capacity={self.capacity}); raise it or use 0 (exact)")

    def candidate_rows(self, t: _Table) -> torch.Tensor:
        if t.rows is None:  # never launched (no data parallel hook): local rows
            t.rows = self._local_rows(t)
            t.notes = []
        return t.rows

    # --------------------------------------------------------------- gradient stats
    def grad_stats(self, flat_grad: torch.Tensor, dense_stats) -> torch.Tensor:
        """[sum g^2, nonfinite] over the dense segments (``dense_stats(view)``) + table rows."""
        out = torch.zeros(2, dtype=torch.float32, device=flat_grad.device)
        pos = 0
        for lo, hi in self.ranges():
            if lo > pos:
                out += dense_stats(flat_grad[pos:lo])
            pos = (hi + 63) // 64 * 64
        if pos < flat_grad.numel():
            out += dense_stats(flat_grad[pos:])
        for t in self.tables.values():
            rows = self.candidate_rows(t)
            if rows.numel():
                g = self.grad2d(t).index_select(0, rows.clamp(min=0).long())
                fin = torch.isfinite(g) | (rows < 0).unsqueeze(1)  # padding rows: ignored
                g = torch.where(rows.unsqueeze(1) >= 0, g, torch.zeros((), dtype=g.dtype, device=g.device))
                out[0] += torch.where(fin, g, torch.zeros_like(g)).pow(2).sum()
                out[1] = torch.maximum(out[1], (~fin).any().float())
        # a step whose distinct rows overflowed the exchange capacity dropped some rows' gradients:
        # flag it like a non-finite gradient, so the optimizer skips it on the device (no update of
        # the rows that WERE exchanged with a partial picture) and check() reports it
        seen = getattr(self, "_overflow_seen", None)
        if seen is None:
            seen = self._overflow_seen = torch.zeros_like(self.overflow)
        out[1] = torch.maximum(out[1], (self.overflow > seen).float())
        seen.copy_(self.overflow)
        out[1] = (out[1] > 0).float()
        return out


def table_names(model: torch.nn.Module, min_rows: int = 0) -> List[str]:
    """The model's embedding tables: 2-D parameters named ``*.embedding`` / ``*.word`` or the
    weight of an ``nn.Embedding`` (``*.embedding.weight``)."""
    out = []
    for n, p in model.named_parameters():
        leaf = n.rsplit(".", 1)[-1]
        is_table = leaf in ("embedding", "word") or n.endswith("embedding.weight")
        if p.requires_grad and p.dim() == 2 and is_table and p.shape[0] >= min_rows:
            out.append(n)
    return out


def note_rows(table: torch.Tensor, ids: torch.Tensor) -> None:
    """Called by ops that gather rows of ``table``: records the ids if the table is sparse."""
    sp = getattr(table, "_pv_sparse", None)
    if sp is not None:
        sp.note(table, ids)

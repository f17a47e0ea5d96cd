"""Training driver: ``fit()`` / ``evaluate()`` / ``train_step()``.

Replaces the reference's ``model.compile("adam", "binary_crossentropy", ["accuracy"])``
+ ``fit_generator(gen, nb_epoch, samples_per_epoch, validation_data, nb_val_samples,
callbacks=[ModelCheckpoint])`` (dssm_cnn_v2/cnn_dssm_th.py:181-206):

* loss modes: ``explicit`` (parity: 1 positive + J negatives, BCE on P(D+|Q)),
  ``in_batch`` (every query vs all docs of the local batch), ``cross_gpu`` (vs all
  docs of all ranks, all-gathered page vectors — the north-star mode);
* metrics with Keras names: ``loss``, ``acc`` (= mean(P > 0.5), Keras binary accuracy
  with y = 1), ``val_loss``, ``val_acc``; ``fit`` returns that ``history`` dict;
* per-epoch checkpoints in the reference layout + final artefacts (io/checkpoint.py);
* resume from the latest checkpoint (step count, optimizer state, RNG, data cursor);
* NaN/inf guard: a non-finite gradient skips the optimizer step on every rank
  (device-side flag, no host sync) and is counted in the metrics;
* fault injection for resume tests: ``PAGEVEC_FAULT_STEP=<n>`` raises at step n.
"""
from __future__ import annotations

import json
import logging
import math
import os
import time
import weakref
from typing import Callable, Dict, Iterable, Iterator, List, Optional, Tuple

import torch

from ..models.base import TwoTowerModel, bump_generation
from ..ops import dense as dops
from ..ops import determinism
from ..ops import grad_sink
from ..ops import loss as lops
from ..ops._common import precision_scope
from ..ops import embedding as eops
from ..ops.optim import FlatAdam, FlatParams, grad_sumsq_and_finite
from ..parallel import dist as pdist
from ..parallel import placement
from ..parallel import sparse_rows, topology
from ..parallel.ddp import GradBuckets, broadcast_params
from ..parallel.sparse_rows import SparseTables
from ..utils.metrics import MetricsLogger, hbm_used_gb
from ..utils.tracing import range_push, range_pop

log = logging.getLogger(__name__)


def _restore_det(prev) -> None:
    """Give the process-wide deterministic mode back as it was before a trainer switched it on."""
    determinism.restore(prev)


# The eager step on a HIGH-priority HIP stream: the query tower (its own stream, models/base.py)
# and the side streams stay at normal priority, so when both towers' backward chains are queued
# the dispatcher feeds the page tower's (the critical path: dense / loss backward -> dTable
# reduce -> dW) first, and the query tower's fills the CUs that are left (round-6 timeline: the
# page tower's small bias column sum waited 110 us behind the query tower's dTable reduce).
STEP_PRIORITY = os.environ.get("PAGEVEC_STEP_PRIORITY", "1") != "0"


class InjectedFault(RuntimeError):
    pass


class PhaseTimer:
    """Step-time breakdown (forward / backward / allreduce / optimizer) for the metrics
    JSONL.  GPU: HIP events, read only when the record is written, so
    the timed steps run without host syncs; CPU: wall clock."""

    PHASES = ("forward", "backward", "allreduce", "optimizer")

    def __init__(self, device: torch.device):
        self.gpu = device.type == "cuda"
        self.marks = []

    def mark(self) -> None:
        if self.gpu:
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            self.marks.append(e)
        else:
            self.marks.append(time.perf_counter())

    def result_ms(self) -> Dict[str, float]:
        if len(self.marks) != len(self.PHASES) + 1:
            return {}
        if self.gpu:
            self.marks[-1].synchronize()
            d = [self.marks[i].elapsed_time(self.marks[i + 1]) for i in range(len(self.PHASES))]
        else:
            d = [1e3 * (self.marks[i + 1] - self.marks[i]) for i in range(len(self.PHASES))]
        out = {f"{p}_ms": round(v, 3) for p, v in zip(self.PHASES, d)}
        out["step_ms"] = round(sum(d), 3)
        return out


class Trainer:
    def __init__(self, cfg, model: TwoTowerModel, device: Optional[torch.device] = None,
                 metrics: Optional[MetricsLogger] = None, graph: bool = False, graph_fence: bool = False):
        self.cfg = cfg
        self.info = pdist.info()
        self.device = device or self.info.device
        self.model = model.to(self.device)
        self.flat = FlatParams(self.model.named_parameters())
        broadcast_params(self.flat)
        bump_generation()
        lazy = None
        if getattr(cfg, "lazy_embedding_adam", False):
            lazy = [n for n, p in self.flat.named if n.rsplit(".", 1)[-1] in ("embedding", "word") and p.dim() == 2]
        # bf16 compute copies written by the optimizer kernel itself (no per-step casts)
        mirror = [n for n in self.model.bf16_mirror_params() if n in self.flat.offsets] \
            if (hasattr(self.model, "bf16_mirror_params") and getattr(cfg, "optimizer_bf16_mirror", True)
                and getattr(cfg, "dtype", "bf16") != "fp32"
                and os.environ.get("PAGEVEC_NO_MIRROR", "0") != "1") else None
        # row-sparse embedding gradients for large vocabularies (parallel/sparse_rows.py)
        self.sparse = (SparseTables(self.flat, sparse_rows.table_names(self.model),
                                    capacity=int(getattr(cfg, "sparse_rows_capacity", -1)))
                       if getattr(cfg, "sparse_embedding_grad", False) else None)
        self.opt = FlatAdam(self.flat, lr=cfg.lr, betas=(cfg.beta1, cfg.beta2), eps=cfg.adam_eps,
                            torch_style=(cfg.model == "bert"), lazy=lazy, mirror=mirror, sparse=self.sparse,
                            warmup=int(getattr(cfg, "lr_warmup_steps", 0)))
        self.placement = getattr(cfg, "placement", "dp")
        if self.placement not in ("dp", "tower"):
            raise ValueError(f"unknown placement {self.placement!r}")
        if self.placement == "tower" and cfg.loss_mode != "explicit":
            raise ValueError("tower placement splits the explicit J-negative slots; use loss_mode=explicit")
        self._replica_checked = False
        self._sink_scanned = set()
        self._pos = {}
        self._acc = None
        # bucket size by xGMI message class (parallel/topology.py; an explicit grad_bucket_mb wins)
        bucket = topology.bucket_mb(topology.grad_mb(self.model), cfg.grad_bucket_mb)
        self.buckets = (GradBuckets(self.flat, bucket, reduce="sum" if self.placement == "tower" else "avg",
                                    sparse=self.sparse)
                        if self.info.enabled else None)
        self.step = 0
        self.epoch = 0
        self.skipped_steps = 0
        self.metrics = metrics
        self._fault_step = int(os.environ.get("PAGEVEC_FAULT_STEP", "-1"))
        self._timer: Optional[PhaseTimer] = None
        # hipGraph mode (single process on a GPU): after GRAPH_WARMUP eager steps the whole
        # step (forward, backward, Adam) is captured once and replayed — one launch per step
        # instead of hundreds (the launch-bound MLP / BERT steps)
        # deterministic reduction mode (ops/determinism.py) is process-wide: it follows the
        # latest Trainer's config; its fixed-point buffer may grow between steps, so no capture
        self.deterministic = bool(getattr(cfg, "deterministic", False))
        # the mode is process-wide: every step of this trainer first puts it in this trainer's
        # state (determinism.ensure), so a deterministic trainer built earlier in the process
        # cannot leak its mode (or its one-stream, no-graph rule) into this one; close() or a
        # finalizer gives the mode back as it was before a deterministic trainer switched it on
        self._det_prev = None
        self._det_fin = None
        if self.deterministic:
            self._det_prev = determinism.set_deterministic(True)
            self._det_fin = weakref.finalize(self, _restore_det, self._det_prev)
        else:
            determinism.ensure(False)
        # data parallel: the collectives are captured with the step (RCCL supports stream
        # capture; the bucket hooks, the page gather and the loss gathers all enqueue on
        # streams that fork from and join back into the capture stream); the sparse tables'
        # fixed-capacity row exchange too, not the exact one (sparse_rows_capacity 0 sizes
        # itself with a host sync); not tower placement
        self.graph_mode = (bool(graph) and self.device.type == "cuda"
                           and (not self.info.enabled or (bool(getattr(cfg, "graph_distributed", False))
                                                          and self.placement == "dp"))
                           and not self.deterministic
                           and (self.sparse is None or self.sparse.capacity != 0))
        # graph_fence: optional device sync after every replay (debugging aid, off by default).
        # Round 1 needed it: replays interleaved with eager allocating work faulted after ~97
        # CDSSM steps inside rocPRIM's onesweep radix sort (the dTable gradient's bucketing),
        # whose ordered-block-id counter and look-back states are reset by hipMemsetAsync
        # nodes inside the captured graph.  The conv backward now sorts with the in-tree
        # radix sort (csrc/kernels/radix_sort.hip: no memsets, no atomics, no look-back) and
        # 300 unfenced replays with a fresh eager batch per step run clean
        # (test_hipgraph_cdssm_unfenced_fresh_batches, docs/PERF.md).
        self.graph_fence = bool(graph_fence)
        self._graph = None
        self._graph_key = None
        self._graph_warm = 0
        self.graph_status = "off" if not self.graph_mode else "pending"
        # optional per-step GPU probes (bench.py): list of (start, before_allreduce_wait,
        # after_allreduce_wait, end) CUDA events per step; replays record (start, end) only
        self.step_events: Optional[list] = None

    def close(self) -> None:
        """Restore the process-wide deterministic mode this trainer switched on (if any)."""
        if self._det_fin is not None:  # a later GC must not restore a stale snapshot
            self._det_fin.detach()
            self._det_fin = None
        if self._det_prev is not None:
            _restore_det(self._det_prev)
            self._det_prev = None

    # ------------------------------------------------------------------ core step
    def _base_seed(self) -> int:
        return (self.cfg.seed * 1000003 + self.step * 7919) & 0x7FFFFFFF

    def compute_loss(self, q_ids: torch.Tensor, d_ids: torch.Tensor, seed: int
                     ) -> Tuple[torch.Tensor, torch.Tensor]:
        """Mean loss over the local batch and per-row P(D+|Q)."""
        with precision_scope(self.cfg):
            return self._compute_loss(q_ids, d_ids, seed)

    def _compute_loss(self, q_ids, d_ids, seed):
        cfg = self.cfg
        B, S, _ = d_ids.shape
        range_push("forward")
        tower = self.placement == "tower" and self.info.enabled
        pre = {}
        if tower and not self._replica_checked:
            self._check_replicated_batch(q_ids, d_ids)
        if tower:  # every rank: same query/head seed; doc slots on their owning ranks
            q, d = placement.placed_forward(self.model, q_ids, d_ids, self._base_seed())
            dn = dops.l2_normalize(d.reshape(B * S, -1))
        else:
            def doc_hook(d_):  # normalise + start the RCCL page gather before the query tower
                pre["dn"] = dops.l2_normalize(d_.reshape(B * S, -1))
                if cfg.loss_mode == "cross_gpu" and self.info.enabled:
                    pre["gather"] = lops.start_page_gather(pre["dn"])
            q, d = self.model(q_ids, d_ids, seed=seed, doc_hook=doc_hook)
            dn = pre["dn"]
        qn = dops.l2_normalize(q)
        clip = bool(getattr(cfg, "cos_clip", True))
        self._acc = None
        if cfg.loss_mode == "explicit":
            per_row, P = lops.dssm_explicit_loss(qn, dn.view(B, S, -1), cfg.GAMMA, clip)
            loss = per_row.mean()
        elif cfg.loss_mode in ("in_batch", "cross_gpu"):
            pos = self._pos_cache(B, S, q.device)
            gamma = float(getattr(cfg, "inbatch_gamma", 0.0) or cfg.GAMMA)
            # mean loss and accuracy straight from the loss kernels (reduce=True)
            if cfg.loss_mode == "cross_gpu" and self.info.enabled:
                loss, P, self._acc = lops.cross_gpu_loss(qn, dn, pos, gamma, clip, gathered=pre.get("gather"),
                                                         reduce=True)
            else:
                loss, P, self._acc = lops.inbatch_loss(qn, dn, pos, gamma, clip, reduce=True)
        else:
            raise ValueError(f"unknown loss_mode {cfg.loss_mode!r}")
        range_pop()
        if tower:  # W identical heads: back-propagate 1/W of each, gradients are SUM-reduced
            loss = placement.scale_grad(loss, 1.0 / self.info.world_size)
        return loss, P

    def _pos_cache(self, B: int, S: int, device) -> torch.Tensor:
        """Positive-document index of each query (row b -> page b*S), built once per shape."""
        key = (B, S, str(device))
        pos = self._pos.get(key)
        if pos is None:
            pos = torch.arange(B, device=device, dtype=torch.int32) * S
            self._pos = {key: pos}
        return pos

    def _check_replicated_batch(self, q_ids: torch.Tensor, d_ids: torch.Tensor) -> None:
        """Tower placement scores this rank's queries against doc slots computed on OTHER
        ranks: all ranks must hold the same batch.  A data-parallel (sharded) loader would
        silently train on mismatched pairs, so the first step compares a checksum of the
        ids over the ranks (one tiny all-reduce, once)."""
        def fp(t: torch.Tensor) -> torch.Tensor:
            x = t.reshape(-1).to(torch.int64)
            w = torch.arange(1, x.numel() + 1, device=x.device, dtype=torch.int64) % 65521 + 1
            return torch.stack([(x * w).sum(), x.sum(), torch.tensor(x.numel(), device=x.device)])
        c = torch.cat([fp(q_ids), fp(d_ids)]).to(self.device).double()
        lo, hi = c.clone(), -c
        pdist.all_reduce_max_(hi)
        pdist.all_reduce_max_(lo)
        if not torch.equal(-hi, c) or not torch.equal(lo, c):
            raise ValueError("placement='tower' needs the SAME batch on every rank (unsharded loader, "
                             "rank-independent seed); got different batches — use placement='dp' for sharded data")
        self._replica_checked = True

    GRAPH_WARMUP = 2

    def train_step(self, q_ids: torch.Tensor, d_ids: torch.Tensor) -> Dict[str, torch.Tensor]:
        # long-bag GEMMs (ops/embedding.py PAGEVEC_BAG_GEMM=auto): the library inside graphs and
        # in the eager steps that warm a capture up (its first call may not happen in a capture),
        # the in-tree kernels for eager-only trainers
        with eops.bag_gemm_scope("lib" if self.graph_mode else None):
            return self._train_step(q_ids, d_ids)

    def _train_step(self, q_ids: torch.Tensor, d_ids: torch.Tensor) -> Dict[str, torch.Tensor]:
        if self.step == self._fault_step:
            raise InjectedFault(f"injected fault at step {self.step}")
        determinism.ensure(self.deterministic)
        if self.graph_mode:
            key = (tuple(q_ids.shape), tuple(d_ids.shape), q_ids.dtype, d_ids.dtype)
            if self._graph is not None and key == self._graph_key:
                return self._replay(q_ids, d_ids)
            if self._graph_warm >= self.GRAPH_WARMUP and self._graph is None:
                if self._capture_agreed(q_ids, d_ids, key):
                    return self._replay(q_ids, d_ids)
                return self._eager_step(q_ids, d_ids)
            self._graph_warm += 1
        return self._prio_step(q_ids, d_ids)

    def priority_stream(self) -> Optional[torch.cuda.Stream]:
        """This trainer's high-priority stream (None when STEP_PRIORITY is off, on the CPU or in
        deterministic mode)."""
        if not (STEP_PRIORITY and self.device.type == "cuda" and not self.deterministic):
            return None
        hp = getattr(self, "_hp_stream", None)
        if hp is None:
            lo, hi = torch.cuda.Stream.priority_range()
            hp = self._hp_stream = torch.cuda.Stream(device=self.device, priority=min(lo, hi))
        return hp

    def stream_context(self):
        """``with trainer.stream_context(): <training loop>`` — the loop's own work (batches,
        metrics) on the high-priority stream too, so consecutive steps need no cross-stream
        hand-off (each hand-off is a queue-to-queue dependency: ~0.2 ms of idle GPU per step
        when the step ran on its own stream and the caller's on the default one)."""
        import contextlib

        hp = self.priority_stream()
        return torch.cuda.stream(hp) if hp is not None else contextlib.nullcontext()

    def _prio_step(self, q_ids: torch.Tensor, d_ids: torch.Tensor) -> Dict[str, torch.Tensor]:
        """The eager step, on this trainer's high-priority stream when STEP_PRIORITY (GPU, not
        deterministic mode, not inside a capture); ordered after and before the caller's stream."""
        hp = self.priority_stream()
        if hp is None or torch.cuda.is_current_stream_capturing():
            return self._eager_step(q_ids, d_ids)
        cur = torch.cuda.current_stream(self.device)
        if cur == hp:  # the caller already runs on it (stream_context)
            return self._eager_step(q_ids, d_ids)
        hp.wait_stream(cur)
        for t in (q_ids, d_ids):
            if t.is_cuda:
                t.record_stream(hp)  # the caller may free its batch while the step still reads it
        with torch.cuda.stream(hp):
            out = self._eager_step(q_ids, d_ids)
        cur.wait_stream(hp)
        for t in out.values():
            if isinstance(t, torch.Tensor) and t.is_cuda:
                t.record_stream(cur)
        return out

    def _capture_agreed(self, q_ids: torch.Tensor, d_ids: torch.Tensor, key) -> bool:
        """Capture the step, then agree on the outcome across ranks (one MIN all-reduce, outside
        any capture): if the capture failed on ANY rank, every rank drops its graph and stays
        eager — a mixed job (some ranks replaying captured collectives, others issuing them
        eagerly in a different order) would deadlock.  The outcome is logged on every rank and
        kept in ``graph_status`` (reported by bench.py)."""
        err = None
        try:
            self._capture(q_ids, d_ids, key)
        except Exception as e:  # noqa: BLE001 - any capture failure falls back to eager
            err = f"{type(e).__name__}: {e}"
            self._graph = None
            if self.device.type == "cuda":
                torch.cuda.synchronize(self.device)
        ok = pdist.all_agree(err is None, self.device)
        if ok:
            self.graph_status = "captured" + (" (dp, RCCL collectives in the graph)" if self.info.enabled else "")
            log.info("rank %d: training step captured in a hipGraph (world %d)", self.info.rank,
                     self.info.world_size)
            return True
        self._graph, self._graph_key = None, None
        self.graph_mode = False
        self.graph_status = "eager (capture failed on " + ("this rank: " + err if err else "another rank") + ")"
        log.warning("rank %d: hipGraph capture abandoned on every rank, eager steps from here: %s", self.info.rank,
                    err or "failed on another rank")
        return False

    # ------------------------------------------------------------------ hipGraph
    def _capture(self, q_ids: torch.Tensor, d_ids: torch.Tensor, key) -> None:
        from ..ops import conv_pool as cops

        self._gq = q_ids.to(self.device).clone()
        self._gd = d_ids.to(self.device).clone()
        self._seed_dev = torch.zeros(1, dtype=torch.int32, device=self.device)
        torch.cuda.synchronize()
        step0, count0 = self.step, self.opt.step_count
        g = torch.cuda.CUDAGraph()
        cops.set_seed_tensor(self._seed_dev)  # conv kernels add the per-replay device seed
        try:
            with torch.cuda.graph(g):
                self._gout = self._eager_step(self._gq, self._gd, seed_override=0, timing=False)
        finally:
            cops.set_seed_tensor(None)
        # the capture only recorded the step: undo its host-side bookkeeping
        self.step, self.opt.step_count = step0, count0
        self._graph, self._graph_key = g, key

    def _event(self) -> torch.cuda.Event:
        e = torch.cuda.Event(enable_timing=True)
        e.record()
        return e

    def _replay(self, q_ids: torch.Tensor, d_ids: torch.Tensor) -> Dict[str, torch.Tensor]:
        e0 = self._event() if self.step_events is not None else None
        self._gq.copy_(q_ids, non_blocking=True)
        self._gd.copy_(d_ids, non_blocking=True)
        seed = (self._base_seed() + self.info.rank * 104729) & 0x7FFFFFFF
        # the captured step ran with seed 0, so every kernel seed was its tower's constant
        # (models/base.py: query 2 s + 1, pages 2 s + 2 + 1000 slot); the kernels add the
        # device value, so 2 s (mod 2^32) replays exactly the eager step's conv-tower dropout
        # masks (BERT derives its layer seeds multiplicatively: fresh, but different, masks)
        d = (2 * seed) & 0xFFFFFFFF
        self._seed_dev.fill_(d - (1 << 32) if d >= (1 << 31) else d)
        self._graph.replay()
        if e0 is not None:
            self.step_events.append((e0, None, None, self._event()))
        if self.graph_fence:
            torch.cuda.synchronize(self.device)
        self.opt.step_count += 1
        self.opt.note_external_step()  # the captured update also rewrote the bf16 mirrors
        bump_generation()
        self.step += 1
        return self._gout

    def _eager_step(self, q_ids: torch.Tensor, d_ids: torch.Tensor, seed_override: Optional[int] = None,
                    timing: bool = True) -> Dict[str, torch.Tensor]:
        self.model.train()
        probe = self.step_events is not None and timing and self.device.type == "cuda"
        ev0 = self._event() if probe else None
        le = self.cfg.log_every
        timer = PhaseTimer(self.device) if (timing and self.metrics and self.metrics.enabled and le and
                                            (self.step + 1) % le == 0) else None
        if timer:
            timer.mark()
        if self.sparse is not None:  # tables: only last step's rows are zeroed
            self.flat.zero_grad(skip=self.sparse.ranges())
            self.sparse.begin_step()
        else:
            self.flat.zero_grad()
        if self.buckets is not None:
            self.buckets.start_step()
        seed = (self._base_seed() + self.info.rank * 104729) & 0x7FFFFFFF
        if seed_override is not None:
            seed = seed_override
        loss, P = self.compute_loss(q_ids, d_ids, seed)
        if timer:
            timer.mark()
        # parameters with several gradient producers keep autograd's accumulation: needed for
        # bucket hooks (DDP) and, on GPU, for towers that share weights across the query side
        # stream and the main stream (a direct write on one stream would race the other's add)
        if (self.buckets is not None and self.buckets.overlap) or self.device.type == "cuda":
            key = (tuple(q_ids.shape), tuple(d_ids.shape))
            if key not in self._sink_scanned:  # once per input shape (ops/grad_sink.py)
                grad_sink.mark_multi_use(loss, self.flat)
                self._sink_scanned.add(key)
        range_push("backward")
        if loss.dim() == 0 and loss.is_cuda:
            # a cached device 1.0 seeds the backward: no fill kernel per step for autograd's
            # implicit ones_like(loss)
            one = getattr(self, "_one", None)
            if one is None or one.device != loss.device or one.dtype != loss.dtype:
                one = self._one = torch.ones((), dtype=loss.dtype, device=loss.device)
            torch.autograd.backward(loss, one)
        else:
            loss.backward()
        range_pop()
        if timer:
            timer.mark()
        range_push("allreduce")
        ev1 = self._event() if probe else None
        if self.buckets is not None:
            self.buckets.finish()
        ev2 = self._event() if probe else None
        range_pop()
        if timer:
            timer.mark()
        range_push("optimizer")
        if self.sparse is not None:
            stats = self.sparse.grad_stats(self.flat.grad, grad_sumsq_and_finite)
        else:
            stats = grad_sumsq_and_finite(self.flat.grad)
        skip = stats[1:2] if self.cfg.skip_nonfinite else None
        self.opt.step(skip)
        if self.sparse is not None:
            self.sparse.finish_step()
        bump_generation()
        range_pop()
        if timer:
            timer.mark()
            self._timer = timer
        if probe:
            self.step_events.append((ev0, ev1, ev2, self._event()))
        self.step += 1
        acc = self._acc if self._acc is not None else (P > 0.5).float().mean()
        return {"loss": loss.detach(), "acc": acc, "grad_sumsq": stats[0],
                "nonfinite": stats[1]}

    @torch.no_grad()
    def eval_step(self, q_ids: torch.Tensor, d_ids: torch.Tensor) -> Dict[str, torch.Tensor]:
        determinism.ensure(self.deterministic)
        self.model.eval()
        loss, P = self.compute_loss(q_ids, d_ids, 0)
        self.model.train()
        return {"loss": loss, "acc": self._acc if self._acc is not None else (P > 0.5).float().mean()}

    # ------------------------------------------------------------------ loops
    def _run_epoch(self, batches: Iterator, steps: int, train: bool) -> Dict[str, float]:
        tot: Dict[str, torch.Tensor] = {}
        n = 0
        t0 = time.perf_counter()
        for _ in range(steps):
            try:
                q, d = next(batches)
            except StopIteration:
                break
            q = q.to(self.device, non_blocking=True)
            d = d.to(self.device, non_blocking=True)
            m = self.train_step(q, d) if train else self.eval_step(q, d)
            for k in ("loss", "acc"):
                tot[k] = tot.get(k, 0.0) + m[k].float()
            if train:
                nf = m["nonfinite"]
                tot["nonfinite"] = tot.get("nonfinite", 0.0) + nf
                if self.sparse is not None and self.cfg.log_every and self.step % self.cfg.log_every == 0:
                    self.sparse.check()  # a host read at the logging cadence: fail early
                if self.metrics and self.cfg.log_every and self.step % self.cfg.log_every == 0:
                    rec = dict(step=self.step, loss=float(m["loss"]), acc=float(m["acc"]),
                               grad_norm=math.sqrt(max(0.0, float(m["grad_sumsq"]))), hbm_gb=round(hbm_used_gb(), 3))
                    if self._timer is not None:
                        rec.update(self._timer.result_ms())
                        if rec.get("step_ms"):
                            rec["pairs_per_s"] = round(q.shape[0] * self.info.world_size * 1e3 / rec["step_ms"], 1)
                        self._timer = None
                    self.metrics.log(**rec)
            n += 1
        if n == 0:
            return {}
        if train and self.sparse is not None:
            self.sparse.check()
        out = {k: float(v) / n for k, v in tot.items() if k != "nonfinite"}
        if train and "nonfinite" in tot:
            self.skipped_steps += int(round(float(tot["nonfinite"])))
        # average metrics over ranks
        if self.info.enabled:
            t = torch.tensor([out.get("loss", 0.0), out.get("acc", 0.0)], device=self.device)
            pdist.all_reduce_mean_(t)
            out["loss"], out["acc"] = float(t[0]), float(t[1])
        out["time_s"] = time.perf_counter() - t0
        out["steps"] = n
        return out

    def fit(self, train_batches: Callable[[int], Iterator], nb_epoch: Optional[int] = None,
            steps_per_epoch: Optional[int] = None, validation_batches: Optional[Callable[[int], Iterator]] = None,
            validation_steps: Optional[int] = None, callbacks: Iterable = ()) -> Dict[str, List[float]]:
        """Keras-style fit. ``train_batches(epoch)`` returns an iterator of (q_ids, d_ids).

        steps_per_epoch defaults to num_train_samples // batch_size (samples_per_epoch).
        """
        cfg = self.cfg
        nb_epoch = nb_epoch or cfg.nb_epoch
        gb = cfg.batch_size
        steps_per_epoch = steps_per_epoch or max(1, cfg.num_train_samples // gb)
        validation_steps = validation_steps or max(1, cfg.num_validation_samples // gb)
        history: Dict[str, List[float]] = {"loss": [], "acc": [], "val_loss": [], "val_acc": []}
        for cb in callbacks:
            if hasattr(cb, "on_train_begin"):
                cb.on_train_begin(self)
        start_epoch = self.epoch
        with self.stream_context():
            self._fit_epochs(train_batches, nb_epoch, steps_per_epoch, validation_batches, validation_steps,
                             callbacks, history, start_epoch)
        for cb in callbacks:
            if hasattr(cb, "on_train_end"):
                cb.on_train_end(self, history)
        return {k: v for k, v in history.items() if v}

    def _fit_epochs(self, train_batches, nb_epoch, steps_per_epoch, validation_batches, validation_steps, callbacks,
                    history, start_epoch) -> None:
        for ep in range(start_epoch, nb_epoch):
            tr = self._run_epoch(iter(train_batches(ep)), steps_per_epoch, True)
            history["loss"].append(tr.get("loss", float("nan")))
            history["acc"].append(tr.get("acc", float("nan")))
            if validation_batches is not None:
                va = self._run_epoch(iter(validation_batches(ep)), validation_steps, False)
                history["val_loss"].append(va.get("loss", float("nan")))
                history["val_acc"].append(va.get("acc", float("nan")))
            self.epoch = ep + 1
            logs = {k: v[-1] for k, v in history.items() if v}
            if self.info.is_main:
                log.info("epoch %d/%d %s", ep + 1, nb_epoch, json.dumps(logs))
            if self.metrics:
                self.metrics.log(epoch=ep + 1, **logs)
            for cb in callbacks:
                if hasattr(cb, "on_epoch_end"):
                    cb.on_epoch_end(self, ep, logs)

    # ------------------------------------------------------------------ state
    def state(self) -> Dict[str, object]:
        return {"step": self.step, "epoch": self.epoch, "skipped_steps": self.skipped_steps,
                "opt_step": self.opt.step_count, "world_size": self.info.world_size}

    def load_state(self, st: Dict[str, object]) -> None:
        self.step = int(st["step"])
        self.epoch = int(st["epoch"])
        self.skipped_steps = int(st.get("skipped_steps", 0))
        self.opt.step_count = int(st.get("opt_step", self.step))
        # the HIP Adam reads its bias corrections from the DEVICE step counter (captured
        # steps replay without the host): it must resume at the same count as the host one
        self.opt.t_dev[0] = float(self.opt.step_count)
        bump_generation()
        self.opt.refresh_mirrors()

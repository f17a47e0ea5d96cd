"""Process-group setup and differentiable collectives (RCCL over xGMI on MI355X).

One process per GPU; ``backend="nccl"`` is RCCL on ROCm.  CPU tests use ``gloo``
(world_size > 1 on one host) — the same code paths.

* ``init_distributed()`` reads RANK / WORLD_SIZE / LOCAL_RANK / MASTER_ADDR / MASTER_PORT
  (torchrun contract), pins the device, sets a finite collective timeout so a hung
  peer surfaces as an error instead of a silent hang.
* ``all_gather_autograd(x)``: forward all-gather of page vectors (cross-GPU in-batch
  negatives); backward = reduce-scatter(sum) of the gathered gradient
  back to the owning rank.  This generic form serves the torch / wide-vector paths; the
  HIP cross-GPU loss (ops/loss.py) instead gathers the queries and scores its LOCAL pages
  against all of them in the backward, so no gradient is reduce-scattered there.
* ``active()``: whether collectives run.  ``PAGEVEC_FORCE_DIST=1`` initialises the process
  group and runs every collective code path even at world size 1 — how the RCCL paths
  (early page gather, async query / scale gathers, bucketed ``ReduceOp.AVG`` all-reduce,
  eager ``device_id`` init) are exercised on a one-GPU box (tests/test_rccl_gpu.py).

The reference has no collectives at all; its only multi-device code is manual tower
placement (dssm_cnn_v2/cnn_dssm_tf.py:139-158), reproduced as ``parallel/placement.py``.
"""
from __future__ import annotations

import datetime
import os
from dataclasses import dataclass
from typing import Optional

import torch
import torch.distributed as dist


@dataclass
class DistInfo:
    rank: int = 0
    world_size: int = 1
    local_rank: int = 0
    backend: str = "none"
    device: torch.device = torch.device("cpu")
    forced: bool = False  # PAGEVEC_FORCE_DIST: collective code paths on at world size 1

    @property
    def is_main(self) -> bool:
        return self.rank == 0

    @property
    def enabled(self) -> bool:
        return self.world_size > 1 or self.forced


def force_requested() -> bool:
    return os.environ.get("PAGEVEC_FORCE_DIST", "0") == "1"


def active(group=None) -> bool:
    """True when the collective code paths run: an initialised process group with more than
    one rank, or any size under PAGEVEC_FORCE_DIST=1."""
    return dist.is_initialized() and (dist.get_world_size(group) > 1 or _INFO.forced)


_INFO = DistInfo()


def info() -> DistInfo:
    return _INFO


def init_distributed(backend: Optional[str] = None, timeout_s: float = 600.0, device: Optional[str] = None) -> DistInfo:
    """Initialise from the torchrun environment; a no-op single-process setup otherwise."""
    global _INFO
    # RCCL's peer-memory IPC on this driver is dmabuf only: the HSA runtime reads this at
    # HIP initialisation, which happens below (set_device) — never earlier in this module
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    use_gpu = (device or ("cuda" if torch.cuda.device_count() > 0 else "cpu")).startswith("cuda")
    if use_gpu:
        torch.cuda.set_device(local % max(1, torch.cuda.device_count()))
        dev = torch.device("cuda", torch.cuda.current_device())
    else:
        dev = torch.device("cpu")
    forced = force_requested()
    if (world > 1 or forced) and not dist.is_initialized():
        # PAGEVEC_DIST_BACKEND=gloo rehearses several ranks on one GPU (RCCL refuses duplicate devices)
        be = backend or os.environ.get("PAGEVEC_DIST_BACKEND") or ("nccl" if use_gpu else "gloo")
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29500")
        kw = {}
        if be == "nccl":
            kw["device_id"] = dev
        dist.init_process_group(be, rank=rank, world_size=world,
                                timeout=datetime.timedelta(seconds=timeout_s), **kw)
        _INFO = DistInfo(rank, world, local, be, dev, forced)
    elif dist.is_initialized():
        _INFO = DistInfo(dist.get_rank(), dist.get_world_size(), local, dist.get_backend(), dev, forced)
    else:
        _INFO = DistInfo(0, 1, 0, "none", dev)
    return _INFO


def set_info(i: DistInfo) -> None:
    global _INFO
    _INFO = i


def barrier() -> None:
    if dist.is_initialized():
        dist.barrier()


def destroy() -> None:
    if dist.is_initialized():
        dist.destroy_process_group()


class _AllGather(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x: torch.Tensor) -> torch.Tensor:
        W = dist.get_world_size()
        x = x.contiguous()
        out = torch.empty((W * x.shape[0],) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
        dist.all_gather_into_tensor(out, x)
        ctx.n = x.shape[0]
        return out

    @staticmethod
    def backward(ctx, g: torch.Tensor) -> torch.Tensor:
        g = g.contiguous()
        out = torch.empty((ctx.n,) + tuple(g.shape[1:]), dtype=g.dtype, device=g.device)
        dist.reduce_scatter_tensor(out, g, op=dist.ReduceOp.SUM)
        return out


def all_gather_autograd(x: torch.Tensor) -> torch.Tensor:
    if not active():
        return x
    return _AllGather.apply(x)


def all_reduce_mean_(t: torch.Tensor) -> torch.Tensor:
    if active():
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        t.div_(dist.get_world_size())
    return t


def all_reduce_max_(t: torch.Tensor) -> torch.Tensor:
    if active():
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return t


def broadcast_(t: torch.Tensor, src: int = 0) -> torch.Tensor:
    if active():
        dist.broadcast(t, src)
    return t


def all_agree(ok: bool, device=None) -> bool:
    """True iff ``ok`` holds on EVERY rank (one MIN all-reduce; the local value on one rank).

    Used where ranks must take the same branch, e.g. the hipGraph capture of a data-parallel
    step: a rank whose capture failed would otherwise replay eagerly while its peers replay
    captured collectives in a different order."""
    if not active():
        return bool(ok)
    dev = device if device is not None else info().device
    t = torch.tensor([1 if ok else 0], dtype=torch.int32, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    return bool(int(t.item()) == 1)


def gather_floats(values, device=None):
    """All ranks' equal-length float lists -> a (world, n) float64 CPU tensor (rank order);
    the local values as a (1, n) tensor without a process group."""
    dev = device if device is not None else info().device
    t = torch.tensor([float(v) for v in values], dtype=torch.float64, device=dev)
    if not active():
        return t.view(1, -1).cpu()
    out = torch.empty(dist.get_world_size() * t.numel(), dtype=torch.float64, device=dev)
    dist.all_gather_into_tensor(out, t)
    return out.view(dist.get_world_size(), -1).cpu()

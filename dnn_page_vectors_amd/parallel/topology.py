"""xGMI topology policy for RCCL: message classes -> bucket size and channel floor.

An MI355X node is 8 GPUs fully connected by point-to-point xGMI: 7 links of ~153 GB/s per GPU,
no switch.  A ring collective moves each byte over ONE link per step, so a single ring is
link-bound at ~153 GB/s; RCCL spreads a collective over several channels (rings / trees, one
workgroup each) to use more links at once.  More channels buy bandwidth for large messages but
each channel is a workgroup taking a CU away from the overlapped backward kernels, and a small
message split over many channels pays per-channel latency instead.

The step's traffic falls in two classes (sizes: SURVEY §2.3 table, ``tools/comm_micro.py``):

* latency class — total gradient <= ``LATENCY_GRAD_MB`` (CDSSM-ngram: 12.6 MB fp32): the
  buckets are cut only where the tower changes (query tower | doc tower | embedding tables),
  so each tower's gradient is ONE collective launched the moment that tower's backward is
  done; no channel floor (RCCL's own small-message tuning), so the overlapped conv backward
  keeps its CUs.
* bandwidth class — larger gradients (MLP 512-512-128: 126 MB, BERT-base: 440 MB): 64 MB
  buckets (several buckets in flight while the backward of earlier layers runs, each large
  enough to keep the channels busy) and a channel floor of ``BANDWIDTH_MIN_CHANNELS`` so that
  every bucket spreads over the node's links (a floor only raises RCCL's default).

Everything is a default: explicit ``NCCL_*`` environment variables and an explicit
``grad_bucket_mb`` win.  The chosen values are reported in bench.py's JSON ``config.comm``;
the per-size channel sweep that tunes these numbers on an 8-GPU node is
``tools/comm_micro.py --sweep-channels``.
"""
from __future__ import annotations

import os
from typing import Dict, Optional

import torch

LATENCY_GRAD_MB = 32.0
BANDWIDTH_BUCKET_MB = 64.0
BANDWIDTH_MIN_CHANNELS = 16
XGMI_LINKS_PER_GPU = 7
# provenance of the three policy constants above: derived from the link arithmetic in the
# module docstring, NOT yet tuned on an 8-GPU node (no node was available to this build; the
# sweep is tools/comm_micro.py --sweep-channels).  Reported with every bench record.
CONSTANTS_STATUS = "unmeasured (derived from xGMI link arithmetic; no 8-GPU sweep yet)"

_APPLIED: Dict[str, str] = {}


def grad_mb(model: torch.nn.Module) -> float:
    return sum(p.numel() for p in model.parameters() if p.requires_grad) * 4 / 2**20


def message_class(total_grad_mb: float) -> str:
    return "latency" if total_grad_mb <= LATENCY_GRAD_MB else "bandwidth"


def bucket_mb(total_grad_mb: float, configured: Optional[float], default: float = 32.0) -> float:
    """The trainer's bucket size: an explicitly configured value (!= the dataclass default)
    wins; otherwise latency class -> one bucket per tower cut, bandwidth class -> 64 MB."""
    if configured is not None and configured != default:
        return float(configured)
    if message_class(total_grad_mb) == "latency":
        return max(total_grad_mb, 1.0) * 2.0  # larger than any tower: only the tower cuts split
    return BANDWIDTH_BUCKET_MB


def apply_env(total_grad_mb: float, world: int) -> Dict[str, str]:
    """Set RCCL environment defaults for this job's class BEFORE the communicator is created
    (``init_process_group`` / first collective).  Returns what was set here."""
    if world <= 1:
        return {}
    if message_class(total_grad_mb) == "bandwidth" and "NCCL_MIN_NCHANNELS" not in os.environ:
        os.environ["NCCL_MIN_NCHANNELS"] = str(BANDWIDTH_MIN_CHANNELS)
        _APPLIED["NCCL_MIN_NCHANNELS"] = str(BANDWIDTH_MIN_CHANNELS)
    return dict(_APPLIED)


def report(total_grad_mb: float, bucket: float) -> Dict[str, object]:
    return {"class": message_class(total_grad_mb), "grad_mb": round(total_grad_mb, 1), "bucket_mb": round(bucket, 1),
            "policy_env": dict(_APPLIED), "xgmi_links_per_gpu": XGMI_LINKS_PER_GPU,
            "policy_constants": {"latency_grad_mb": LATENCY_GRAD_MB, "bandwidth_bucket_mb": BANDWIDTH_BUCKET_MB,
                                 "bandwidth_min_channels": BANDWIDTH_MIN_CHANNELS, "status": CONSTANTS_STATUS}}

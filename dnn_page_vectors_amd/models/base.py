"""Two-tower model base class.

Every model maps token ids to vectors with a *query tower* and a *document tower*
(reference: ``query_model = model(Lq)``, ``doc_model = model(Ld)``, the doc tower
shared by the positive and the J negatives, dssm_cnn_v2/cnn_dssm_th.py:147-156).

Subclasses implement ``tower_forward(tower, ids, training, seed)``.  The base
class provides ``forward`` (raw tower outputs for a training batch), ``encode``
(L2-normalised vectors, no dropout; the page-vector extraction API the reference
never had — its only pattern is reading weights, old_scripts/simple_rnn.py:51) and
the compute-cache refresh hook used after optimizer steps.
"""
from __future__ import annotations

import os
from typing import Dict, Optional, Tuple

import torch
import torch.nn as nn

from ..ops import dense as dops
from ..ops import determinism
from ..ops._common import precision_scope

# hipGraph captures keep the query tower / early-sort side streams (the capture forks into them
# and joins back; round 6): graph steps MLP 1.148 -> 1.078 ms, chunked fp8 1.047 ->
# 0.997, chunked CDSSM 1.125 -> 1.048 (profiles/r6/capture_streams_ab.txt).  The round-5 segfault
# in capture_end came from a fork of a fork — the query tower's early sort on a side stream of
# the query stream — which conv_pool._capture_streams keeps out of captures.  0: one stream.
CAPTURE_STREAMS = os.environ.get("PAGEVEC_CAPTURE_STREAMS", "1") != "0"
# cuda_stream handles of the query-tower streams (a fork of the capture stream inside a capture)
QUERY_STREAM_IDS = set()

_GENERATION = [0]


def bump_generation() -> None:
    """Invalidate derived compute copies (bf16 tables, packed weights) of all models."""
    _GENERATION[0] += 1


class TwoTowerModel(nn.Module):
    def __init__(self, cfg):
        super().__init__()
        self.cfg = cfg
        self._cache_gen = -1
        self._cache: Dict[str, object] = {}

    # ---- to implement ----------------------------------------------------------
    def tower_forward(self, tower: str, ids: torch.Tensor, training: bool, seed: int,
                      slot: int = 0) -> torch.Tensor:  # pragma: no cover - abstract
        raise NotImplementedError

    @property
    def out_dim(self) -> int:  # pragma: no cover - abstract
        raise NotImplementedError

    def build_cache(self) -> Dict[str, object]:
        """Derived low-precision copies of the parameters used by the fused kernels."""
        return {}

    def bf16_mirror_params(self):
        """Names of parameters whose bf16 copy the optimizer should write with each update
        (ops/optim.py::mirror_for); default none."""
        return []

    # ---- shared ------------------------------------------------------------------
    def compute_cache(self) -> Dict[str, object]:
        if self._cache_gen != _GENERATION[0] or not self._cache:
            with torch.no_grad():
                self._cache = self.build_cache()
            self._cache_gen = _GENERATION[0]
        return self._cache

    def forward(self, q_ids: torch.Tensor, d_ids: torch.Tensor, seed: int = 0, doc_hook=None
                ) -> Tuple[torch.Tensor, torch.Tensor]:
        """q_ids (B, Lq); d_ids (B, S, Ld) with S = 1+J docs per query (positive first).

        Returns raw (unnormalised) q (B, D) and d (B, S, D).  The doc tower runs FIRST and
        ``doc_hook(d)`` is called before the query tower, so a cross-GPU page gather can be
        in flight while the query tower computes.
        """
        with precision_scope(self.cfg):
            return self._forward(q_ids, d_ids, seed, doc_hook)

    def _forward(self, q_ids, d_ids, seed, doc_hook):
        B, S, Ld = d_ids.shape
        training = self.training
        side = self._query_stream(q_ids)
        if getattr(self.cfg, "share_doc_tower", True):
            d = self.tower_forward("doc", d_ids.reshape(B * S, Ld), training, seed * 2 + 2).view(B, S, -1)
        else:  # v1: independent towers per document slot (dssm_cnn/cnn_dssm.py:160-164)
            d = torch.stack([self.tower_forward("doc", d_ids[:, s], training, seed * 2 + 2 + 1000 * s, slot=s)
                             for s in range(S)], dim=1)
        if doc_hook is not None:
            doc_hook(d)
        if side is None:
            q = self.tower_forward("query", q_ids, training, seed * 2 + 1)
            return q, d
        # The query tower on a side stream: autograd runs each backward op on the stream of
        # its forward op, so the query tower's backward (its own sparse conv backward, sort,
        # dense GEMMs) overlaps the page tower's on the main stream; the engine joins the
        # streams before backward() returns.
        main = torch.cuda.current_stream(q_ids.device)
        side.wait_stream(main)
        q_ids.record_stream(side)
        with torch.cuda.stream(side):
            q = self.tower_forward("query", q_ids, training, seed * 2 + 1)
        main.wait_stream(side)
        q.record_stream(main)
        return q, d

    def _query_stream(self, q_ids: torch.Tensor) -> Optional[torch.cuda.Stream]:
        if not (q_ids.is_cuda and self.training and getattr(self.cfg, "query_stream", False)):
            return None
        if os.environ.get("PAGEVEC_QUERY_STREAM", "1") == "0":  # A/B switch
            return None
        if torch.cuda.is_current_stream_capturing() and not CAPTURE_STREAMS:  # hipGraph capture: one stream
            return None
        if determinism.enabled():  # deterministic mode: one stream (ops/determinism.py)
            return None
        if self._towers_share_params():
            # a tied parameter would get the query tower's gradient written on the side
            # stream (grad sink) and the page tower's added by autograd on the main stream:
            # nothing orders the two, so shared towers keep one stream
            return None
        st = getattr(self, "_qstreams", None)
        if st is None:
            st = self._qstreams = {}
        dev = q_ids.device.index
        if dev not in st:
            st[dev] = torch.cuda.Stream(device=q_ids.device)
            QUERY_STREAM_IDS.add(st[dev].cuda_stream)
        return st[dev]

    def _towers_share_params(self) -> bool:
        """True when the query tower and a page tower hold the same parameter object
        (siamese BERT on the unpacked path, any tied weight); computed once."""
        v = getattr(self, "_towers_shared", None)
        if v is None:
            q = getattr(self, "query_tower", None)
            docs = list(getattr(self, "doc_towers", []) or [])
            qp = {id(p) for p in q.parameters()} if q is not None else set()
            v = any(id(p) in qp for d in docs for p in d.parameters())
            self._towers_shared = v
        return v

    @torch.no_grad()
    def encode(self, ids: torch.Tensor, tower: str = "doc", batch_size: int = 4096,
               normalize: bool = True) -> torch.Tensor:
        """Vectors for ``ids`` (N, L) from one tower, evaluated without dropout."""
        was = self.training
        self.eval()
        outs = []
        try:
            with torch.no_grad(), precision_scope(self.cfg):  # no autograd graph: nothing saved
                for i in range(0, ids.shape[0], batch_size):
                    v = self.tower_forward(tower, ids[i:i + batch_size], False, 0)
                    outs.append(dops.l2_normalize(v) if normalize else v)
        finally:
            self.train(was)
        return torch.cat(outs, 0) if outs else torch.empty(0, self.out_dim, device=ids.device)

    def architecture(self) -> Dict[str, object]:
        """JSON-able description (the cnn_dssm_model_only.json analogue)."""
        return {"class": type(self).__name__, "config": self.cfg.to_dict(),
                "params": {n: list(p.shape) for n, p in self.named_parameters()}}

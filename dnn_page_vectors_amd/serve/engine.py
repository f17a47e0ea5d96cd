"""Encoder engine with dynamic batching — text in, page / query vectors out.

Serving requests arrive one or a few texts at a time; the GPU wants thousands of rows
per launch (the fused conv kernel runs a persistent grid over the batch).  The engine
therefore queues requests and a single worker thread drains the queue into batches of
up to ``max_batch`` texts (or whatever arrived within ``max_wait_ms``), runs the native
C++ featurizer once per batch, one ``model.encode`` per tower, and resolves each
request's future with its slice.  One worker thread owns the device (no concurrent
launches from request threads); request threads only wait.

``encode(texts, tower)`` is the synchronous API; ``submit`` returns a Future.
"""
from __future__ import annotations

import queue
import threading
import time
from concurrent.futures import Future
from typing import List, Optional, Sequence, Tuple

import numpy as np
import torch


class EncoderEngine:
    def __init__(self, model, featurizer, query_length: int, document_length: int,
                 device: Optional[torch.device] = None, max_batch: int = 4096, max_wait_ms: float = 2.0):
        self.model = model
        self.fz = featurizer
        self.lengths = {"query": int(query_length), "doc": int(document_length)}
        self.device = device or next(model.parameters()).device
        self.max_batch = int(max_batch)
        self.max_wait = float(max_wait_ms) / 1e3
        self._q: "queue.Queue[Tuple[str, List[str], Future]]" = queue.Queue()
        self._stop = threading.Event()
        self.batches = 0
        self.texts = 0
        self._worker = threading.Thread(target=self._run, name="pagevec-encoder", daemon=True)
        self._worker.start()

    # ------------------------------------------------------------------ client API
    def submit(self, texts: Sequence[str], tower: str = "doc") -> Future:
        if tower not in self.lengths:
            raise ValueError("tower must be 'query' or 'doc'")
        fut: Future = Future()
        if not texts:
            fut.set_result(torch.empty(0, self.model.out_dim))
            return fut
        self._q.put((tower, list(texts), fut))
        return fut

    def encode(self, texts: Sequence[str], tower: str = "doc", timeout: Optional[float] = 60.0) -> torch.Tensor:
        """L2-normalised fp32 vectors (len(texts), D) on the CPU."""
        return self.submit(texts, tower).result(timeout=timeout)

    def close(self) -> None:
        self._stop.set()
        self._q.put(("", [], Future()))  # wake the worker
        self._worker.join(timeout=10)

    # ------------------------------------------------------------------ worker
    def _collect(self) -> List[Tuple[str, List[str], Future]]:
        first = self._q.get()
        reqs = [first]
        n = len(first[1])
        deadline = time.monotonic() + self.max_wait
        while n < self.max_batch:
            left = deadline - time.monotonic()
            if left <= 0:
                break
            try:
                r = self._q.get(timeout=left)
            except queue.Empty:
                break
            reqs.append(r)
            n += len(r[1])
        return reqs

    def _run(self) -> None:
        while not self._stop.is_set():
            reqs = [r for r in self._collect() if r[1]]
            if not reqs:
                continue
            for tower in ("query", "doc"):
                group = [r for r in reqs if r[0] == tower]
                if not group:
                    continue
                try:
                    texts = [t for r in group for t in r[1]]
                    vec = self._encode_batch(texts, tower)
                    off = 0
                    for _, t, fut in group:
                        fut.set_result(vec[off:off + len(t)])
                        off += len(t)
                except Exception as e:  # deliver the failure to every waiting request
                    for _, _, fut in group:
                        if not fut.done():
                            fut.set_exception(e)

    @torch.no_grad()
    def _encode_batch(self, texts: List[str], tower: str) -> torch.Tensor:
        L = self.lengths[tower]
        ids = np.empty((len(texts), L), dtype=np.int32)
        self.fz(texts, L, out=ids)
        t = torch.from_numpy(ids).to(self.device, non_blocking=False)
        vec = self.model.encode(t, tower, batch_size=self.max_batch).float().cpu()
        self.batches += 1
        self.texts += len(texts)
        return vec


__all__ = ["EncoderEngine"]

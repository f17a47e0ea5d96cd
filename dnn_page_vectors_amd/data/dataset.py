"""JSONL pair datasets and the prefetching batch loader (L4 input pipeline).

Reference: ``DataHelpers.load_data_generator`` (dssm_cnn_v2/data_helpers.py:128-197) reads
``{'q', 'doc_corr', 'doc_incorr'[J]}`` lines sequentially, featurizes every row in Python
and ``np.vstack``s them (O(B^2) copies), then yields ``([q, pos, neg_1..neg_J], ones)``.

Here:
* ``JsonlPairDataset`` mmaps the file once in C++ (csrc/runtime/featurize.cpp), indexes
  the valid rows (rows with != J negatives are skipped, as the reference does) and
  featurizes any set of rows with a thread pool straight into int32 buffers;
* ``PairLoader`` turns a dataset (or the synthetic generator) into an epoch iterator:
  sequential order by default (reference semantics) or a seeded per-epoch shuffle, a
  rank shard for data parallelism, a background thread that keeps ``prefetch`` batches
  featurized in pinned host memory, and non-blocking H2D copies; its cursor
  (epoch, batch) is part of the checkpoint so a resumed run continues where it stopped.
"""
from __future__ import annotations

import ctypes
import queue
import threading
from typing import Iterator, Optional, Tuple

import numpy as np
import torch

from .. import _native
from .featurize import Featurizer
from .text import MODES


class JsonlPairDataset:
    def __init__(self, path: str, featurizer: Featurizer, query_length: int, document_length: int,
                 num_negatives: int = 3, nthreads: int = 0):
        self.path = path
        self.fz = featurizer
        self.qlen, self.dlen, self.J = int(query_length), int(document_length), int(num_negatives)
        self.nthreads = nthreads or featurizer.nthreads
        self._lib = _native.runtime()
        self._h = self._lib.pv_dataset_open(path.encode(), self.J, self.nthreads)
        if not self._h:
            raise FileNotFoundError(path)

    def __len__(self) -> int:
        return int(self._lib.pv_dataset_size(self._h))

    @property
    def skipped(self) -> int:
        return int(self._lib.pv_dataset_skipped(self._h))

    def close(self) -> None:
        if getattr(self, "_h", None):
            self._lib.pv_dataset_close(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def batch(self, rows: np.ndarray, q_out: Optional[np.ndarray] = None, d_out: Optional[np.ndarray] = None
              ) -> Tuple[np.ndarray, np.ndarray]:
        rows = np.ascontiguousarray(rows, dtype=np.int64)
        n = rows.shape[0]
        if q_out is None:
            q_out = np.empty((n, self.qlen), dtype=np.int32)
        if d_out is None:
            d_out = np.empty((n, 1 + self.J, self.dlen), dtype=np.int32)
        rc = self._lib.pv_dataset_batch(self._h, rows.ctypes.data, n, self.fz.native_mode, self.qlen, self.dlen,
                                        self.fz.handle(), self.fz.hash_size, self.fz.unk_id, self.fz.pad_id,
                                        q_out.ctypes.data, d_out.ctypes.data, self.nthreads)
        if rc != 0:
            raise RuntimeError(f"pv_dataset_batch failed: {rc}")
        return q_out, d_out

    def texts(self, row: int):
        """[q, doc_corr, *doc_incorr] of one row (decoded by the native parser)."""
        out = []
        for field in range(2 + self.J):
            n = self._lib.pv_dataset_row_text(self._h, row, field, None, 0)
            buf = ctypes.create_string_buffer(int(n) + 1)
            self._lib.pv_dataset_row_text(self._h, row, field, buf, int(n) + 1)
            out.append(buf.raw[:n].decode("utf-8"))
        return out


class PairLoader:
    """Epoch iterator of (q_ids, d_ids) torch batches with background prefetch."""

    def __init__(self, dataset: JsonlPairDataset, batch_size: int, shuffle: bool = False, seed: int = 1337,
                 rank: int = 0, world_size: int = 1, prefetch: int = 2, device: Optional[torch.device] = None,
                 drop_last: bool = True, pin_memory: Optional[bool] = None):
        self.ds = dataset
        self.B = int(batch_size)
        self.shuffle = shuffle
        self.seed = seed
        self.rank, self.world = rank, world_size
        self.prefetch = max(1, prefetch)
        self.device = device
        self.drop_last = drop_last
        self.pin = (device is not None and device.type == "cuda") if pin_memory is None else pin_memory
        self.epoch = 0
        self.cursor = 0  # batches already consumed in the current epoch

    def order(self, epoch: int) -> np.ndarray:
        n = len(self.ds)
        if self.shuffle:
            return np.random.default_rng(self.seed + epoch).permutation(n)
        return np.arange(n)

    def num_batches(self) -> int:
        per_rank = len(self.ds) // self.world
        return per_rank // self.B if self.drop_last else -(-per_rank // self.B)

    def _rank_rows(self, epoch: int) -> np.ndarray:
        o = self.order(epoch)
        per_rank = len(o) // self.world
        return o[self.rank * per_rank:(self.rank + 1) * per_rank]

    def state(self) -> dict:
        return {"epoch": self.epoch, "cursor": self.cursor}

    def load_state(self, st: dict) -> None:
        self.epoch, self.cursor = int(st["epoch"]), int(st["cursor"])

    def epoch_iter(self, epoch: Optional[int] = None, fresh: bool = False) -> Iterator[Tuple[torch.Tensor, torch.Tensor]]:
        """Batches of ``epoch`` from the saved cursor (resume); ``fresh``: from its first batch
        (validation passes, whose consumer may stop before the end)."""
        if fresh or (epoch is not None and epoch != self.epoch):
            self.epoch, self.cursor = (self.epoch if epoch is None else epoch), 0
        rows = self._rank_rows(self.epoch)
        nb = self.num_batches()
        start = self.cursor
        q: "queue.Queue" = queue.Queue(maxsize=self.prefetch)
        stop = threading.Event()

        def work():
            try:
                for b in range(start, nb):
                    if stop.is_set():
                        return
                    r = rows[b * self.B:(b + 1) * self.B]
                    qa = torch.empty((len(r), self.ds.qlen), dtype=torch.int32, pin_memory=self.pin)
                    da = torch.empty((len(r), 1 + self.ds.J, self.ds.dlen), dtype=torch.int32, pin_memory=self.pin)
                    self.ds.batch(r, qa.numpy(), da.numpy())
                    q.put((qa, da))
                q.put(None)
            except Exception as e:  # surface worker errors in the consumer
                q.put(e)

        t = threading.Thread(target=work, daemon=True)
        t.start()
        try:
            while True:
                item = q.get()
                if item is None:
                    break
                if isinstance(item, Exception):
                    raise item
                qa, da = item
                if self.device is not None:
                    qa = qa.to(self.device, non_blocking=True)
                    da = da.to(self.device, non_blocking=True)
                self.cursor += 1
                yield qa, da
        finally:
            stop.set()
            while t.is_alive():
                try:
                    q.get_nowait()
                except queue.Empty:
                    t.join(timeout=0.05)
        self.epoch += 1
        self.cursor = 0


class SyntheticLoader:
    """Same interface over ``data.synthetic.SyntheticPairs`` (device-side generation)."""

    def __init__(self, gen, batch_size: int, steps_per_epoch: int):
        self.gen, self.B, self.steps = gen, batch_size, steps_per_epoch
        self.epoch = 0
        self.cursor = 0

    def state(self) -> dict:
        return {"epoch": self.epoch, "cursor": self.cursor}

    def load_state(self, st: dict) -> None:
        self.epoch, self.cursor = int(st["epoch"]), int(st["cursor"])

    def epoch_iter(self, epoch: Optional[int] = None, fresh: bool = False):
        # a consumer that stops after exactly ``steps`` batches never runs the epilogue below:
        # a new epoch index (or fresh) restarts the cursor, as in PairLoader (without it every
        # other epoch of a CLI run was empty)
        if fresh or (epoch is not None and epoch != self.epoch):
            self.epoch, self.cursor = (self.epoch if epoch is None else epoch), 0
        for _ in range(self.cursor, self.steps):
            self.cursor += 1
            yield self.gen.batch(self.B)
        self.epoch += 1
        self.cursor = 0


class InMemoryPairs:
    """The v1 data path (dssm_cnn/data_helpers.py:261-307 + cnn_dssm.py:201): the
    whole JSONL file featurized into memory once, every field padded to the DATASET's longest
    text (``pad_sentences`` pads to the max length, :88-103) — capped here by the configured
    lengths, which the reference left unbounded — and Keras ``fit(validation_split=s,
    shuffle=True)`` semantics: the LAST ``s`` fraction of the rows (file order) is the
    validation set, the training rows are re-shuffled every epoch (``batch_iter``, :310-324).

    ``train_loader`` / ``val_loader`` give the ``epoch_iter`` interface of ``PairLoader``
    (device tensors, resumable cursor)."""

    def __init__(self, path: str, featurizer: Featurizer, query_length: int, document_length: int,
                 num_negatives: int = 3, validation_split: float = 0.2, nthreads: int = 0):
        if not 0.0 <= validation_split < 1.0:
            raise ValueError("validation_split must be in [0, 1)")
        ds = JsonlPairDataset(path, featurizer, query_length, document_length, num_negatives, nthreads)
        try:
            n = len(ds)
            q, d = ds.batch(np.arange(n))
            self.skipped = ds.skipped
        finally:
            ds.close()
        pad = featurizer.pad_id

        def used(x: np.ndarray) -> int:  # longest non-padding prefix over all rows
            nz = (x != pad).reshape(-1, x.shape[-1])
            if not nz.any():
                return 1
            last = x.shape[-1] - np.argmax(nz[:, ::-1], axis=1)
            return int(np.max(np.where(nz.any(axis=1), last, 0)))

        self.query_length, self.document_length = used(q), used(d)
        self.q = torch.from_numpy(np.ascontiguousarray(q[:, :self.query_length]))
        self.d = torch.from_numpy(np.ascontiguousarray(d[:, :, :self.document_length]))
        # Keras fit(validation_split=s): split_at = int(n * (1 - s)); rows [split_at, n) validate
        self.n_train = int(n * (1.0 - validation_split))
        self.n_val = n - self.n_train

    def __len__(self) -> int:
        return self.n_train + self.n_val

    def train_loader(self, batch_size: int, shuffle: bool = True, seed: int = 1337,
                     device: Optional[torch.device] = None, rank: int = 0, world_size: int = 1,
                     drop_last: bool = False) -> "_TensorLoader":
        """Keras fit semantics: the last partial batch is trained on (``drop_last=False``)."""
        return _TensorLoader(self.q[:self.n_train], self.d[:self.n_train], batch_size, shuffle, seed, device, rank,
                             world_size, drop_last)

    def val_loader(self, batch_size: int, device: Optional[torch.device] = None, rank: int = 0,
                   world_size: int = 1, drop_last: bool = False) -> "_TensorLoader":
        return _TensorLoader(self.q[self.n_train:], self.d[self.n_train:], batch_size, False, 0, device, rank,
                             world_size, drop_last)


class _TensorLoader:
    """Batches of in-memory (q, d) tensors; per-epoch seeded shuffle; rank shard; cursor."""

    def __init__(self, q: torch.Tensor, d: torch.Tensor, batch_size: int, shuffle: bool, seed: int,
                 device: Optional[torch.device], rank: int, world_size: int, drop_last: bool = False):
        self.q, self.d, self.B = q, d, int(batch_size)
        self.drop_last = bool(drop_last)
        self.shuffle, self.seed, self.device = shuffle, seed, device
        self.rank, self.world = rank, world_size
        self.epoch = 0
        self.cursor = 0

    def num_batches(self) -> int:
        per = self.q.shape[0] // self.world  # every rank gets the same number of rows
        return per // self.B if self.drop_last else (per + self.B - 1) // self.B

    def state(self) -> dict:
        return {"epoch": self.epoch, "cursor": self.cursor}

    def load_state(self, st: dict) -> None:
        self.epoch, self.cursor = int(st["epoch"]), int(st["cursor"])

    def epoch_iter(self, epoch: Optional[int] = None, fresh: bool = False) -> Iterator[Tuple[torch.Tensor, torch.Tensor]]:
        if fresh or (epoch is not None and epoch != self.epoch):
            self.epoch, self.cursor = (self.epoch if epoch is None else epoch), 0
        n = self.q.shape[0]
        order = (np.random.default_rng(self.seed + self.epoch).permutation(n) if self.shuffle else np.arange(n))
        per = n // self.world
        order = torch.from_numpy(order[self.rank * per:(self.rank + 1) * per])
        for b in range(self.cursor, self.num_batches()):
            idx = order[b * self.B:(b + 1) * self.B]
            qa, da = self.q[idx], self.d[idx]
            if self.device is not None:
                qa, da = qa.to(self.device, non_blocking=True), da.to(self.device, non_blocking=True)
            self.cursor += 1
            yield qa, da
        self.epoch += 1
        self.cursor = 0

"""Featurizer front-end over the native C++ runtime (``csrc/runtime/featurize.cpp``).

Replaces the per-row Python tokenisation + ``np.vstack`` loop of the
reference generator (``dssm_cnn_v2/data_helpers.py:161-192``), which is
O(B^2) in copies, with one multithreaded native call per batch that writes
straight into a (pinned) int32 buffer.
"""
from __future__ import annotations

import ctypes
import json
import os
from typing import Iterable, List, Optional, Sequence

import numpy as np

from .. import _native
from .text import MODES, PAD, Vocab, build_vocab_counts, normalize_html_line, split_features

HTML_FLAG = 4  # mode bit of the native calls: HTML / word2vec normalisation first


class Featurizer:
    """text -> int32 ids of fixed length ([HTML-normalise,] clean, split, cutoff, pad, lookup/hash).

    ``html=True`` (``Configuration.html_normalize``) runs the reference's page-text normaliser
    (utils/word2vec_normalizer.py:116-146: unescape, strip tags, dot / punctuation rules) on
    every text before ``clean_str`` — natively, inside the same multithreaded call."""

    def __init__(self, mode: str = "char", vocab: Optional[Vocab] = None, hash_size: int = 0,
                 nthreads: int = 0, html: bool = False):
        if mode not in MODES:
            raise ValueError(f"mode must be one of {list(MODES)}")
        if hash_size <= 1 and vocab is None:
            raise ValueError("Featurizer needs a vocab or hash_size > 1")
        self.mode = mode
        self.html = bool(html)
        self.vocab = vocab
        self.hash_size = hash_size if hash_size > 1 else 0
        self.nthreads = nthreads or min(16, os.cpu_count() or 4)
        self._lib = _native.runtime()
        self._vh = None
        if self.hash_size == 0:
            self._vh = self._lib.pv_vocab_new()
            for i, t in enumerate(vocab.itos):
                self._lib.pv_vocab_add(self._vh, t.encode("utf-8"), i)

    @property
    def num_ids(self) -> int:
        return self.hash_size if self.hash_size else len(self.vocab)

    @property
    def pad_id(self) -> int:
        return 0

    @property
    def unk_id(self) -> int:
        return 1

    def __del__(self):
        if getattr(self, "_vh", None):
            try:
                self._lib.pv_vocab_free(self._vh)
            except Exception:
                pass

    def __call__(self, texts: Sequence[str], length: int, out: Optional[np.ndarray] = None) -> np.ndarray:
        n = len(texts)
        if out is None:
            out = np.empty((n, length), dtype=np.int32)
        assert out.dtype == np.int32 and out.shape == (n, length) and out.flags.c_contiguous
        if n == 0:
            return out
        enc = [t.encode("utf-8") for t in texts]
        arr = (ctypes.c_char_p * n)(*enc)
        rc = self._lib.pv_featurize(arr, n, self.native_mode, length, self._vh, self.hash_size,
                                    self.unk_id, self.pad_id, out.ctypes.data, self.nthreads)
        if rc != 0:
            raise RuntimeError(f"pv_featurize failed: {rc}")
        return out

    def handle(self):
        return self._vh

    @property
    def native_mode(self) -> int:
        return MODES[self.mode] | (HTML_FLAG if self.html else 0)


def clean_str_native(s: str) -> str:
    lib = _native.runtime()
    b = s.encode("utf-8")
    cap = 4 * len(b) + 16
    buf = ctypes.create_string_buffer(cap)
    n = lib.pv_clean_str(b, buf, cap)
    return buf.raw[:n].decode("utf-8")


def normalize_html_native(s: str) -> str:
    """data/text.py::normalize_html_line through the C++ featurizer (parity tests)."""
    lib = _native.runtime()
    b = s.encode("utf-8")
    n = lib.pv_normalize_html(b, None, 0)
    buf = ctypes.create_string_buffer(int(n) + 1)
    lib.pv_normalize_html(b, buf, int(n) + 1)
    return buf.raw[:n].decode("utf-8")


def iter_jsonl_texts(path: str, num_neg: int) -> Iterable[List[str]]:
    """[q, doc_corr, *doc_incorr] per valid row (rows with != num_neg negatives skipped)."""
    with open(path, encoding="utf-8") as f:
        for line in f:
            line = line.strip()
            if not line:
                continue
            d = json.loads(line)
            if len(d.get("doc_incorr", [])) != num_neg:
                continue
            yield [d["q"], d["doc_corr"]] + list(d["doc_incorr"])


def generate_vocabulary(files: Sequence[str], mode: str, num_neg: int, html: bool = False) -> Vocab:
    """Vocabulary over train+val files (dssm_cnn_v2/data_helpers.py:77-124), no cutoff.

    Deterministic: reserved tokens first, then by descending count, ties lexicographic.
    ``html``: tokens of the HTML-normalised text (the featurizer's ``html=True`` input).
    """
    from collections import Counter

    c: Counter = Counter()
    for fn in files:
        for texts in iter_jsonl_texts(fn, num_neg):
            for t in texts:
                c.update(split_features(normalize_html_line(t) if html else t, mode))
    toks = [w for w, _ in sorted(c.items(), key=lambda kv: (-kv[1], kv[0])) if w != PAD]
    return Vocab(toks)


__all__ = ["Featurizer", "clean_str_native", "normalize_html_native", "generate_vocabulary", "iter_jsonl_texts", "build_vocab_counts"]

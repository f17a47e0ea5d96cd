"""Pretrained word-vector ingestion (fastText ``.vec`` / word2vec text).

Reference: ``load_word_embeddings_compact`` (dssm_cnn_v2/data_helpers.py:17-74): parse
whitespace-separated lines, skip lines shorter than ``embedding_dim`` fields, keep the
first ``embedding_dim`` floats of words present in the vocabulary, and draw rows for
unseen words from U(-0.25, 0.25).  Output is the (V, E) init matrix for the embedding
table, cached as safetensors (the reference pickled it with joblib).
"""
from __future__ import annotations

import os
from typing import Optional, Tuple

import numpy as np
import torch

from ..data.text import Vocab


def load_word_vectors(path: str, vocab: Vocab, dim: int, seed: int = 1337,
                      limit: Optional[int] = None) -> Tuple[np.ndarray, int]:
    """Returns (weights (len(vocab), dim) float32, number of vocab words found)."""
    rng = np.random.default_rng(seed)
    W = rng.uniform(-0.25, 0.25, size=(len(vocab), dim)).astype(np.float32)
    found = 0
    with open(path, "r", encoding="utf-8", errors="replace") as f:
        for n, line in enumerate(f):
            if limit is not None and n >= limit:
                break
            parts = line.rstrip().split()
            if len(parts) < dim + 1:
                continue  # header line "count dim" or short/garbled line
            i = vocab.stoi.get(parts[0])
            if i is None:
                continue
            try:
                W[i] = np.asarray(parts[1:dim + 1], dtype=np.float32)
                found += 1
            except ValueError:
                continue
    W[vocab.pad_id] = 0.0
    return W, found


def cached_word_vectors(cfg, vocab: Vocab) -> np.ndarray:
    from safetensors.numpy import load_file, save_file

    path = cfg.embedding_weights_file_tpl.format(cfg.masking_value)
    if cfg.embeddings_pickled and os.path.exists(path):
        return load_file(path)["weights"]
    W, _ = load_word_vectors(cfg.word_vectors_file, vocab, cfg.embedding_dim, cfg.seed)
    if cfg.create_data_dump:
        os.makedirs(os.path.dirname(path), exist_ok=True)
        save_file({"weights": W}, path)
    return W


def init_embedding_(param: torch.nn.Parameter, W: np.ndarray) -> None:
    with torch.no_grad():
        param.copy_(torch.from_numpy(W).to(param.device, param.dtype))

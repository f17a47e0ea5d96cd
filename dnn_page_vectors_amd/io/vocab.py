"""Vocabulary persistence (the reference joblib-pickled ``vocab_set_{m}.pkl`` /
``vocab_index_dict_{m}.pkl``, dssm_cnn_v2/data_helpers.py:120-123, become JSON)."""
from __future__ import annotations

import json
import os

from ..data.text import Vocab
from ..utils.fs import create_dir


def save_vocab(vocab: Vocab, cfg) -> str:
    create_dir(cfg.pickle_files_dir)
    path = cfg.vocab_index_file.format(cfg.masking_value)
    with open(path + ".tmp", "w", encoding="utf-8") as f:
        json.dump(vocab.to_json(), f, ensure_ascii=False)
    os.replace(path + ".tmp", path)
    with open(cfg.vocab_set_file.format(cfg.masking_value), "w", encoding="utf-8") as f:
        json.dump(sorted(vocab.itos), f, ensure_ascii=False)
    return path


def load_vocab(cfg) -> Vocab:
    with open(cfg.vocab_index_file.format(cfg.masking_value), encoding="utf-8") as f:
        return Vocab.from_json(json.load(f))

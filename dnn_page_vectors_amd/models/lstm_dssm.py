"""Legacy LSTM two-tower model (reference old_scripts/lstm.py:125-200, lstm_new.py:136-246).

Tower: Embedding(V, 100, mask_zero) -> Dropout(0.25) -> [optional Conv1D(64, 3, relu) ->
MaxPool(2), lstm_new.py] -> LSTM(64) (last state over the non-padded prefix) -> Dense(32,
relu).  The reference wires five independent towers into ``Merge(mode='cos') -> 1 - x ->
concat -> Dense(4, softmax)`` trained with categorical cross-entropy on all-ones labels
(a defect); here the towers feed the same cosine gamma-softmax head as every
other model.  Recurrent cells run on MIOpen through torch.nn.LSTM (low priority legacy
path).
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..parallel.sparse_rows import note_rows

from .base import TwoTowerModel


class LSTMTower(nn.Module):
    def __init__(self, vocab_size: int, E: int, hidden: int, dense: int, conv: bool, p: float):
        super().__init__()
        self.embedding = nn.Embedding(vocab_size, E, padding_idx=0)
        nn.init.uniform_(self.embedding.weight, -0.05, 0.05)
        self.conv = nn.Conv1d(E, 64, 3) if conv else None
        self.lstm = nn.LSTM(64 if conv else E, hidden, batch_first=True)
        self.dense = nn.Linear(hidden, dense)
        self.p = p

    def forward(self, ids: torch.Tensor, training: bool) -> torch.Tensor:
        ids = ids.long()
        note_rows(self.embedding.weight, ids)  # sparse-gradient tables (parallel/sparse_rows.py)
        x = F.dropout(self.embedding(ids), self.p, training)
        lengths = (ids != 0).sum(1).clamp(min=1)
        if self.conv is not None:
            x = F.max_pool1d(torch.relu(self.conv(x.transpose(1, 2))), 2).transpose(1, 2)
            lengths = ((lengths - 2).clamp(min=1) // 2).clamp(min=1, max=x.shape[1])
        packed = nn.utils.rnn.pack_padded_sequence(x, lengths.cpu(), batch_first=True, enforce_sorted=False)
        _, (h, _) = self.lstm(packed)
        return torch.relu(self.dense(h[-1]))


class LSTMDSSM(TwoTowerModel):
    def __init__(self, cfg, vocab_size: int):
        super().__init__(cfg)
        torch.manual_seed(int(cfg.seed))
        mk = lambda: LSTMTower(vocab_size, cfg.embedding_dim, cfg.lstm_output_size, cfg.lstm_dense_units,
                               getattr(cfg, "lstm_conv", False), float(cfg.dropout_prob[0]))
        self.vocab_size = vocab_size
        self.query_tower = mk()
        self.doc_towers = nn.ModuleList([mk() for _ in range(1 if cfg.share_doc_tower else 1 + cfg.J)])

    @property
    def out_dim(self) -> int:
        return self.cfg.lstm_dense_units

    def tower_forward(self, tower: str, ids: torch.Tensor, training: bool, seed: int, slot: int = 0) -> torch.Tensor:
        if tower == "query":
            return self.query_tower(ids, training)
        return self.doc_towers[slot if len(self.doc_towers) > 1 else 0](ids, training)

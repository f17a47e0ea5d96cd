"""Model zoo: every model is a two-tower ``TwoTowerModel`` (models/base.py)."""
from __future__ import annotations


def build_model(cfg, vocab_size: int):
    """Instantiate the model named by ``cfg.model``."""
    name = cfg.model
    if name == "cdssm":
        from .cdssm import CDSSM

        return CDSSM(cfg, vocab_size)
    if name == "mlp":
        from .mlp_dssm import MLPDSSM

        return MLPDSSM(cfg, vocab_size)
    if name == "bert":
        from .bert_dual import BertDualEncoder

        return BertDualEncoder(cfg, vocab_size)
    if name == "chunked":
        from .chunked import ChunkedPageEncoder

        return ChunkedPageEncoder(cfg, vocab_size)
    if name == "lstm":
        from .lstm_dssm import LSTMDSSM

        return LSTMDSSM(cfg, vocab_size)
    raise KeyError(f"unknown model {name!r}")


MODELS = ["cdssm", "mlp", "bert", "chunked", "lstm"]

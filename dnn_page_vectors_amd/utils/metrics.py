"""Per-step / per-epoch metrics as JSON lines.

The reference only printed Keras ``hist.history`` (cnn_dssm_th.py:196).  Here every
record is one JSON object per line with a wall-clock timestamp; rank 0 writes.
"""
from __future__ import annotations

import json
import os
import time
from typing import Any, Optional


class MetricsLogger:
    def __init__(self, path: Optional[str], enabled: bool = True):
        self.path = path
        self.enabled = enabled and path is not None
        if self.enabled:
            os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)

    def log(self, **kw: Any) -> None:
        if not self.enabled:
            return
        kw.setdefault("ts", time.time())
        with open(self.path, "a") as f:
            f.write(json.dumps(kw, sort_keys=True) + "\n")

    def read(self):
        if not self.path or not os.path.exists(self.path):
            return []
        with open(self.path) as f:
            return [json.loads(l) for l in f if l.strip()]


def hbm_used_gb() -> float:
    try:
        import torch

        if torch.cuda.is_available():
            return torch.cuda.max_memory_allocated() / 1e9
    except Exception:
        pass
    return 0.0

"""HTTP serving front-end (FastAPI): encode texts, index pages, search by query text.

    python -m dnn_page_vectors_amd serve --preset cdssm_ngram_bf16 --weights model.safetensors \
        [--pages pages.jsonl] [--index idx] --host 127.0.0.1 --port 8000

Endpoints (JSON):
  GET  /health                         {"status", "pages", "device", "batches", "texts"}
  POST /encode   {"texts": [...], "tower": "doc"|"query"}      -> {"vectors": [[...]], "dim"}
  POST /index/add {"pages": [{"id": ..., "text": ...}]}        -> {"added", "pages"}
  POST /search   {"queries": [...], "k": 10}                   -> {"results": [[{"id", "score"}]]}
  POST /index/save {"name": ...}                               -> {"saved", "pages"}
       (only when the server was started with a save directory, ``--save-dir``: the name is
       a plain file stem resolved inside that directory; anything that would escape it is
       rejected — the HTTP client never chooses a filesystem path)

Every list in a request body is capped (``max_items``, default 4096 texts / pages / queries)
and every text is capped at ``max_chars`` characters, so one request cannot make the
engine featurize and encode an unbounded batch.

Request handlers run in FastAPI's thread pool and only wait on the engine's futures:
all device work goes through the EncoderEngine worker (dynamic batching) and the index
search, serialised by a lock so one HIP stream sees a well-ordered launch sequence.
"""
from __future__ import annotations

import os
import re
import threading
from typing import Any, List, Optional, Union

from pydantic import BaseModel, Field

from .engine import EncoderEngine
from .index import PageIndex


# request bodies (module level: FastAPI resolves the handlers' annotations by name)
class EncodeReq(BaseModel):
    texts: List[str]
    tower: str = "doc"


class Page(BaseModel):
    id: Union[int, str]
    text: str


class AddReq(BaseModel):
    pages: List[Page]


class SearchReq(BaseModel):
    queries: List[str]
    k: int = Field(10, ge=1)


class SaveReq(BaseModel):
    name: str


_NAME = re.compile(r"^[A-Za-z0-9][A-Za-z0-9_.-]{0,127}$")


def resolve_save_path(save_dir: str, name: str) -> str:
    """``save_dir/name`` for a plain file stem; ValueError for anything else (separators,
    ``..``, absolute paths, hidden names) or a result outside ``save_dir``."""
    if not _NAME.match(name) or ".." in name:
        raise ValueError(f"invalid index name {name!r}: use [A-Za-z0-9_.-], no path separators")
    root = os.path.realpath(save_dir)
    path = os.path.realpath(os.path.join(root, name))
    if os.path.dirname(path) != root:
        raise ValueError(f"index name {name!r} escapes the save directory")
    return path


def create_app(engine: EncoderEngine, index: PageIndex, max_k: int = 100, save_dir: Optional[str] = None,
               max_items: int = 4096, max_chars: int = 100_000):
    """``save_dir``: directory that POST /index/save writes into (None: the endpoint is off).
    ``max_items`` / ``max_chars``: per-request caps on list length and text length."""
    from fastapi import FastAPI, HTTPException

    app = FastAPI(title="dnn_page_vectors_amd", version="1")
    lock = threading.Lock()

    def _cap(texts: List[str]) -> None:
        if len(texts) > max_items:
            raise HTTPException(413, f"at most {max_items} items per request")
        if any(len(t) > max_chars for t in texts):
            raise HTTPException(413, f"texts are limited to {max_chars} characters")

    @app.get("/health")
    def health() -> Any:
        return {"status": "ok", "pages": len(index), "device": str(index.device), "batches": engine.batches,
                "texts": engine.texts}

    @app.post("/encode")
    def encode(req: EncodeReq) -> Any:
        if req.tower not in ("doc", "query"):
            raise HTTPException(400, "tower must be 'doc' or 'query'")
        _cap(req.texts)
        v = engine.encode(req.texts, req.tower)
        return {"vectors": v.tolist(), "dim": int(v.shape[1]) if v.dim() == 2 else 0}

    @app.post("/index/add")
    def add(req: AddReq) -> Any:
        if not req.pages:
            return {"added": 0, "pages": len(index)}
        _cap([p.text for p in req.pages])
        v = engine.encode([p.text for p in req.pages], "doc")
        with lock:
            index.add(v, [p.id for p in req.pages], normalize=False)
            n = len(index)
        return {"added": len(req.pages), "pages": n}

    @app.post("/search")
    def search(req: SearchReq) -> Any:
        if req.k > max_k:
            raise HTTPException(400, f"k must be <= {max_k}")
        if not req.queries:
            return {"results": []}
        _cap(req.queries)
        q = engine.encode(req.queries, "query")
        with lock:
            hits = index.search(q, req.k)
        return {"results": [[{"id": i, "score": s} for i, s in row] for row in hits]}

    @app.post("/index/save")
    def save(req: SaveReq) -> Any:
        if save_dir is None:
            raise HTTPException(403, "index saving is disabled (start the server with --save-dir)")
        try:
            path = resolve_save_path(save_dir, req.name)
        except ValueError as e:
            raise HTTPException(400, str(e))
        with lock:
            index.save(path)
            n = len(index)
        return {"saved": os.path.basename(path), "pages": n}

    return app


def build_service(cfg, weights: Optional[str] = None, device=None, max_batch: int = 4096, max_wait_ms: float = 2.0,
                  index_path: Optional[str] = None):
    """Model (+ weights) + featurizer + engine + index for a configuration."""
    import torch

    from ..cli import _featurizer
    from ..io import checkpoint as ck
    from ..models import build_model

    dev = torch.device(device) if device else torch.device("cuda" if torch.cuda.device_count() > 0 else "cpu")
    fz = _featurizer(cfg)
    model = build_model(cfg, fz.num_ids).to(dev)
    if weights:
        ck.load_weights(model, weights)
    model.eval()
    engine = EncoderEngine(model, fz, cfg.query_length, cfg.document_length, dev, max_batch, max_wait_ms)
    index = PageIndex.load(index_path, device=dev) if index_path else PageIndex(model.out_dim, device=dev)
    return engine, index


__all__ = ["create_app", "build_service"]

"""Serving: page-vector index (HBM-resident, HIP top-k), dynamic-batching encoder engine,
HTTP front-end (``python -m dnn_page_vectors_amd serve``)."""
from .engine import EncoderEngine
from .index import PageIndex, ShardedPageIndex

__all__ = ["EncoderEngine", "PageIndex", "ShardedPageIndex"]

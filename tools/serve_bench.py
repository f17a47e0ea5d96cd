"""Serving micro-benchmark (1 GPU): page-index search latency / throughput and the
dynamic-batching encoder engine under concurrent clients.

    python tools/serve_bench.py [--pages 1000000] [--dim 150]

* search: N random unit page vectors resident in HBM (bf16 padded rows), query batches of
  1 / 64 / 1024, k = 10, HIP top-k kernel (ops/topk.py::topk_cos_padded);
* engine: CDSSM-300d (random init, hashed trigrams, query 45 / page 2000 tokens),
  C client threads each sending single-text requests; reports texts/s and batches formed.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pages", type=int, default=1_000_000)
    ap.add_argument("--dim", type=int, default=150)
    ap.add_argument("--clients", type=int, default=64)
    ap.add_argument("--requests", type=int, default=40)
    a = ap.parse_args()
    from dnn_page_vectors_amd.serve.index import PageIndex

    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    idx = PageIndex(a.dim, device=dev, capacity=a.pages)
    for s in range(0, a.pages, 1 << 18):
        n = min(1 << 18, a.pages - s)
        idx.add(torch.randn(n, a.dim, device=dev, generator=g))
    for B in (1, 64, 1024):
        q = torch.randn(B, a.dim, device=dev, generator=g)
        idx.search_rows(q, 10)
        torch.cuda.synchronize()
        it = 20 if B < 1024 else 5
        t0 = time.perf_counter()
        for _ in range(it):
            idx.search_rows(q, 10)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / it
        print(json.dumps({"search": {"pages": a.pages, "batch": B, "ms": round(dt * 1e3, 3),
                                     "queries_per_s": round(B / dt, 1),
                                     "page_scores_per_s": round(B * a.pages / dt / 1e9, 2)}}), flush=True)

    from dnn_page_vectors_amd.config import preset_config
    from dnn_page_vectors_amd.data.featurize import Featurizer
    from dnn_page_vectors_amd.models import build_model
    from dnn_page_vectors_amd.serve.engine import EncoderEngine

    cfg = preset_config("cdssm_ngram_bf16")
    fz = Featurizer("ngram", hash_size=cfg.vocab_hash_size)
    model = build_model(cfg, cfg.vocab_hash_size).to(dev).eval()
    eng = EncoderEngine(model, fz, cfg.query_length, cfg.document_length, dev, max_batch=4096, max_wait_ms=2.0)
    words = ["statue", "liberty", "new", "york", "tour", "ticket", "museum", "harbor", "ferry", "island"]
    for tower, n_words in (("query", 4), ("doc", 300)):
        texts = [" ".join(words[(i * 7 + j) % len(words)] for j in range(n_words)) + f" {i}"
                 for i in range(a.clients * a.requests)]
        eng.encode(texts[:64], tower)  # warm up
        b0, t_0 = eng.batches, eng.texts

        def client(c):
            for r in range(a.requests):
                eng.encode([texts[c * a.requests + r]], tower)

        th = [threading.Thread(target=client, args=(c,)) for c in range(a.clients)]
        t0 = time.perf_counter()
        for t in th:
            t.start()
        for t in th:
            t.join()
        dt = time.perf_counter() - t0
        n = eng.texts - t_0
        print(json.dumps({"engine": {"tower": tower, "clients": a.clients, "texts": n, "s": round(dt, 3),
                                     "texts_per_s": round(n / dt, 1), "batches": eng.batches - b0,
                                     "mean_batch": round(n / max(1, eng.batches - b0), 1)}}), flush=True)
    eng.close()


if __name__ == "__main__":
    main()

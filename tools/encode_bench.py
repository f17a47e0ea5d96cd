"""Page-vector extraction throughput (encode(), the serving path): pages/s of
``model.encode(ids, "doc")`` — fused gather -> conv -> max-pool -> dense -> L2-normalise
without dropout — on device-resident synthetic pages, random-init weights, 1 GPU.

    python tools/encode_bench.py [--model cdssm|mlp|bert|cdssm_char] [--pages 65536] [--batch 16384]
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from dnn_page_vectors_amd.config import preset_config
    from dnn_page_vectors_amd.data.synthetic import SyntheticPairs, spec_from_config
    from dnn_page_vectors_amd.models import build_model

    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="cdssm", choices=["cdssm", "mlp", "bert", "cdssm_char"])
    ap.add_argument("--pages", type=int, default=65536)
    ap.add_argument("--batch", type=int, default=16384)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--dtype", default=None, choices=["bf16", "fp32"], help="override the preset's dtype "
                    "(reference_char is fp32: the fp32-MFMA conv kernels)")
    a = ap.parse_args()
    preset = {"cdssm": "cdssm_ngram_bf16", "mlp": "mlp_xgpu", "bert": "bert_dp8", "cdssm_char": "reference_char"}[a.model]
    cfg = preset_config(preset)
    if a.model == "cdssm_char":
        cfg = cfg.replace(vocab_hash_size=100)
    if a.dtype:
        cfg = cfg.replace(dtype=a.dtype)
    if a.model == "bert":
        a.pages, a.batch = min(a.pages, 4096), min(a.batch, 1024)
    dev = torch.device("cuda")
    V = cfg.vocab_hash_size
    model = build_model(cfg, V).to(dev)
    data = SyntheticPairs(spec_from_config(cfg, V, num_pages=a.pages), dev, seed=3)
    _, pages = data.eval_set(a.pages)
    ids = pages.reshape(-1, pages.shape[-1])[: a.pages].contiguous()
    model.encode(ids[: a.batch], "doc", batch_size=a.batch)  # warm-up (caches, kernels)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.iters):
        out = model.encode(ids, "doc", batch_size=a.batch)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / a.iters
    print(json.dumps({"model": a.model, "dtype": cfg.dtype, "pages": int(ids.shape[0]), "page_len": int(ids.shape[1]),
                      "dim": int(out.shape[1]), "batch": a.batch, "ms": round(1e3 * dt, 3),
                      "pages_per_s": round(ids.shape[0] / dt, 1),
                      "tokens_per_s": round(ids.numel() / dt), "norm_check": round(float(out[0].norm()), 4)}),
          flush=True)


if __name__ == "__main__":
    main()

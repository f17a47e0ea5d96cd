"""Recall@10 spread of the headline recipe: 1000 fresh-batch steps of CDSSM-300d (B 4096,
cross-GPU loss on one rank) per (data seed, deterministic mode) — the noise band the
tests/test_kernels_gpu.py::test_cdssm_recall_quality_guard threshold has to sit below.

    python tools/recall_spread.py --seeds 1337 2024 --det 0 1 [--steps 1000]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from dnn_page_vectors_amd.config import preset_config  # noqa: E402
from dnn_page_vectors_amd.data.synthetic import SyntheticPairs, spec_from_config  # noqa: E402
from dnn_page_vectors_amd.eval.retrieval import recall_at_k  # noqa: E402
from dnn_page_vectors_amd.models import build_model  # noqa: E402
from dnn_page_vectors_amd.ops import determinism  # noqa: E402
from dnn_page_vectors_amd.parallel import dist as pdist  # noqa: E402
from dnn_page_vectors_amd.train.trainer import Trainer  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seeds", type=int, nargs="+", default=[1337])
    ap.add_argument("--det", type=int, nargs="+", default=[0])
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--set", nargs="*", default=[])
    a = ap.parse_args()
    dev = torch.device("cuda")
    pdist.set_info(pdist.DistInfo(device=dev))
    for det in a.det:
        for seed in a.seeds:
            cfg = preset_config("cdssm_ngram_bf16").override(a.set).replace(deterministic=bool(det))
            model = build_model(cfg, cfg.vocab_hash_size)
            tr = Trainer(cfg, model, dev)
            data = SyntheticPairs(spec_from_config(cfg, cfg.vocab_hash_size, num_pages=65536), dev, seed=seed)
            for _ in range(a.steps):
                m = tr.train_step(*data.batch(cfg.batch_size))
            qe, pe = data.eval_set(2048)
            with torch.no_grad():
                r = recall_at_k(model.encode(qe, "query"), model.encode(pe, "doc"), torch.arange(2048, device=dev),
                                k=10)
            print(json.dumps({"seed": seed, "deterministic": det, "steps": a.steps, "loss": round(float(m["loss"]), 4),
                              "recall_at_10": round(float(r), 4)}), flush=True)
            tr.close()
    determinism.set_deterministic(False)


if __name__ == "__main__":
    main()

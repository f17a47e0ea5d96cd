"""Fraction of ReLU-dead (sample, filter) pairs of the CDSSM conv towers during training (their
dTable sort keys are the dead sentinel V): measures how much of the 17.2 M-entry page-tower
sort a live-only compaction would remove.

    python tools/dead_pairs_probe.py [--steps 300]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=300)
    a = ap.parse_args()
    from dnn_page_vectors_amd.config import preset_config
    from dnn_page_vectors_amd.data.synthetic import SyntheticPairs, spec_from_config
    from dnn_page_vectors_amd.models import build_model
    from dnn_page_vectors_amd.ops import conv_pool as cp
    from dnn_page_vectors_amd.train.trainer import Trainer

    cfg = preset_config("cdssm_ngram_bf16")
    dev = torch.device("cuda")
    V = cfg.vocab_hash_size
    tr = Trainer(cfg, build_model(cfg, V), dev, graph=False)
    data = SyntheticPairs(spec_from_config(cfg, V, num_pages=65536), dev, seed=1337)
    rec = []
    orig = cp.conv_relu_maxpool_fused

    def wrapped(ids, *args, **kw):
        out = orig(ids, *args, **kw)
        pooled = out[0] if isinstance(out, tuple) else out
        rec.append((ids.shape[1], float((pooled.detach() <= 0).float().mean())))
        return out
    cp.conv_relu_maxpool_fused = wrapped
    out = {}
    for s in range(a.steps):
        rec.clear()
        tr.train_step(*data.batch(cfg.batch_size))
        if s in (0, 10, 50, 100, 200, a.steps - 1):
            torch.cuda.synchronize()
            out[s] = {f"L{L}": round(f, 3) for L, f in rec}
    print(json.dumps(out))


if __name__ == "__main__":
    main()

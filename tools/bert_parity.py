"""BERT (config 4) parity arm at full depth: the same initial 12-layer model trained on the same
batches through the HIP step (bf16 MFMA, fused kernels) and through eager fp32 PyTorch ops;
prints one JSON line with both loss curves' head / tail and Recall@10 on held-out pairs.

    python tools/bert_parity.py [--layers 12] [--batch 64] [--steps 200] [--lr 2e-5] [--set k=v ...]

The tests' 2-layer arm (tests/test_kernels_gpu.py::test_new_config_training_curve_hip_matches_torch)
is the fast regression; this is the full-depth run VERDICT r4 #7 asks for before tuning the preset.
"""
import argparse
import copy
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layers", type=int, default=12)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--pages", type=int, default=4096)
    ap.add_argument("--eval", type=int, default=1024)
    ap.add_argument("--set", action="append", default=[])
    a = ap.parse_args()
    from dnn_page_vectors_amd.config import preset_config
    from dnn_page_vectors_amd.data.synthetic import SyntheticPairs, spec_from_config
    from dnn_page_vectors_amd.eval.retrieval import recall_at_k
    from dnn_page_vectors_amd.models import build_model
    from dnn_page_vectors_amd.parallel import dist as pdist
    from dnn_page_vectors_amd.train.trainer import Trainer

    dev = torch.device("cuda")
    pdist.set_info(pdist.DistInfo(device=dev))
    base = preset_config("bert_dp8").replace(bert_layers=a.layers, batch_size=a.batch)
    if a.set:
        base = base.override(a.set)
    V = base.vocab_hash_size
    torch.manual_seed(21)
    m0 = build_model(base, V)
    torch.backends.cudnn.enabled = False
    res = {"layers": a.layers, "batch": a.batch, "steps": a.steps, "overrides": a.set, "lr": base.lr}
    for dtype in ("bf16", "fp32"):
        cfg = base.replace(dtype=dtype)
        model = copy.deepcopy(m0)
        model.cfg = cfg
        tr = Trainer(cfg, model, dev)
        data = SyntheticPairs(spec_from_config(cfg, V, num_pages=a.pages), dev, seed=77)
        t0 = time.time()
        losses = []
        for i in range(a.steps):
            losses.append(float(tr.train_step(*data.batch(cfg.batch_size))["loss"]))
            if i % 50 == 0:
                print(f"{dtype} step {i}: loss {losses[-1]:.4f}", file=sys.stderr, flush=True)
        qe, pe = data.eval_set(a.eval)
        with torch.no_grad():
            r = recall_at_k(model.encode(qe, "query"), model.encode(pe, "doc"), torch.arange(a.eval, device=dev), k=10)
        k = max(10, a.steps // 6)
        res[dtype] = {"loss0": round(losses[0], 4), "tail": round(sum(losses[-k:]) / k, 4),
                      "curve_every_20": [round(x, 3) for x in losses[::20]], "recall_at_10": round(r, 4),
                      "wall_s": round(time.time() - t0, 1)}
        del tr, model
        torch.cuda.empty_cache()
    b, f = res["bf16"], res["fp32"]
    res["tail_rel_diff"] = round(abs(b["tail"] - f["tail"]) / f["tail"], 4)
    res["recall_diff"] = round(abs(b["recall_at_10"] - f["recall_at_10"]), 4)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
